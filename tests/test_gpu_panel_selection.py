"""K04 at panel scale on the GPU (csrc/dgp.hip sel_gen_count / sel_gen_flags /
sel_gen_mark): the device selection over generated rows equals data/selection.py's
transform (``ate_replication.Rmd:97-121``) applied to the SAME device-generated values,
the kept panel rows are those rows, and the DML estimate on the selected bf16 panel sits
within a hundredth of an SE of the float64 panel of the same kept rows."""
import numpy as np
import pytest
import torch

from ate_replication_causalml_amd.data import dgp
from ate_replication_causalml_amd.data.device_dgp import fold_slices, synthetic_panel
from ate_replication_causalml_amd.data.panel_selection import kept_gids, plan_selection
from ate_replication_causalml_amd.data.selection import drop_indices

pytestmark = pytest.mark.gpu


def _device_rows(n, gpu, seed):
    """The first n generated rows of the tutorial model, unselected (the rule's draws in
    fp64, the rest in fp32)."""
    return synthetic_panel(n, p=21, folds=1, seed=seed, dtype="f64", device=gpu,
                           dgp="tutorial-rct")


@pytest.mark.parametrize("compat", ["reference", "textbook"])
def test_device_selection_equals_host_transform(gpu, compat):
    N, seed = 36000, 21                    # ~2e5 generated rows (keep fraction ~0.18)
    sel = plan_selection(N, seed, dgp.TUTORIAL, device=gpu, compat=compat)
    assert sel.n_gen > 150000
    full = _device_rows(sel.n_gen, gpu, seed)
    Xc = full.colmajor()[:, :sel.n_gen].cpu().numpy()
    X = Xc[1:22].T                                   # 15 cts + sex + 5 history
    W = Xc[full.cols["W"]]
    drop = drop_indices(X, W, dgp.COVARIATES, compat=compat)
    keep = np.ones(sel.n_gen, dtype=bool)
    keep[drop] = False
    want = np.flatnonzero(keep)
    got = kept_gids(sel, [(0, N)], device=gpu).cpu().numpy()
    assert len(want) == N
    assert np.array_equal(got, want)
    # the selected panel stores exactly those rows (same draws)
    pan = synthetic_panel(N, p=21, folds=5, seed=seed, dtype="f64", device=gpu, dgp="tutorial",
                          selection=sel, compat=compat)
    m = (pan.row_index >= 0).cpu()
    rows = pan.row_index.cpu()[m]
    Xp = pan.colmajor().cpu()[:, m]
    assert torch.equal(Xp, torch.from_numpy(Xc[:, got[rows.numpy()]]))


def test_cpu_and_gpu_panels_keep_the_same_rows(gpu):
    """The selection rule's draws are fp64 on both sides (csrc/dgp.hip core_draws /
    dgp_normal_d, the formulas of data/dgp.py selection_flags without FMA contraction), so a
    CPU panel (host flags) and a GPU panel (device flags) of the same (N, seed) analyse the
    SAME df_mod: equal n_generated, thresholds, per-block counts and kept rows at N = 2e5,
    seed 21; the stored rule columns (yob, city: fp64 panels) agree to the last few ulps of
    log / cos, the vote history and W exactly."""
    N, seed = 200_000, 21
    sg = plan_selection(N, seed, dgp.TUTORIAL, device=gpu)
    sc = plan_selection(N, seed, dgp.TUTORIAL, device="cpu")
    assert (sg.n_gen, sg.thr_t, sg.thr_c, sg.cand_t, sg.cand_c) == \
        (sc.n_gen, sc.thr_t, sc.thr_c, sc.cand_t, sc.cand_c)
    for f in ("blk_ct", "blk_cc", "blk_kept"):
        np.testing.assert_array_equal(getattr(sg, f), getattr(sc, f))
    kg = kept_gids(sg, [(0, N)], device=gpu).cpu().numpy()
    kc = kept_gids(sc, [(0, N)]).numpy()
    np.testing.assert_array_equal(kg, kc)
    n = 30_000
    pg = synthetic_panel(n, p=21, folds=5, seed=seed, dtype="f64", device=gpu, dgp="tutorial")
    pc = synthetic_panel(n, p=21, folds=5, seed=seed, dtype="f64", device="cpu", dgp="tutorial")
    np.testing.assert_array_equal(pg.gen_ids.cpu().numpy(), pc.gen_ids.numpy())
    Xg, Xc = pg.colmajor().cpu().numpy(), pc.colmajor().numpy()
    for c in ("x0", "x1"):                                  # yob, city
        j = pg.cols[c]
        np.testing.assert_allclose(Xg[j], Xc[j], rtol=1e-13, atol=1e-13)
    for c in ["W"] + [f"x{16 + k}" for k in range(5)]:      # W and the vote history
        np.testing.assert_array_equal(Xg[pg.cols[c]], Xc[pc.cols[c]])


def test_device_selection_sharded_slices(gpu):
    """Kept-rank slices of 3 ranks (kernel path, blocks that start and end mid-slice)
    reassemble the world-1 kept set."""
    N = 20000
    sel = plan_selection(N, 5, dgp.TUTORIAL, device=gpu)
    ref = kept_gids(sel, [(0, N)], device=gpu).cpu().numpy()
    got = np.full(N, -1, dtype=np.int64)
    for r in range(3):
        sl = fold_slices(N, 5, r, 3)
        g = kept_gids(sel, sl, device=gpu).cpu().numpy()
        o = 0
        for a, c in sl:
            got[a:a + c] = g[o:o + c]
            o += c
    assert np.array_equal(got, ref)


def test_dml_tutorial_bf16_vs_f64_parity(gpu):
    """The confounded panel: bf16 storage moves the DML ATE by < 0.05 SE (the bench's
    parity block reports the same ratio at N = 1e7)."""
    from ate_replication_causalml_amd.estimators.lasso import dml_crossfit_panel
    sel = plan_selection(200000, 2, dgp.TUTORIAL, device=gpu)
    pb = synthetic_panel(200000, p=60, folds=5, seed=2, dtype="bf16", device=gpu, dgp="tutorial",
                         selection=sel)
    p64 = synthetic_panel(200000, p=60, folds=5, seed=2, dtype="f64", device=gpu, dgp="tutorial",
                          selection=sel)
    rb = dml_crossfit_panel(pb, 5)[0].cpu().numpy()
    r64 = dml_crossfit_panel(p64, 5)[0].cpu().numpy()
    assert np.isfinite(rb).all() and np.isfinite(r64).all()
    assert abs(rb[0] - r64[0]) < 0.05 * r64[1]
    assert abs(rb[1] - r64[1]) < 0.02 * r64[1]
