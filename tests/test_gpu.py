"""GPU numerics tests: every HIP kernel against a plain float64 PyTorch/numpy
reference of the same op, and every device estimator against the float64 CPU
reference path (T-ref). Run on the MI355X box: ``pytest -m gpu``."""
import numpy as np
import pytest
import torch

from ate_replication_causalml_amd import _native
from ate_replication_causalml_amd.ops import gram as gram_op
from ate_replication_causalml_amd.ops import stats as S
from ate_replication_causalml_amd.ops.linalg import chol_solve, logistic_irls, predict
from ate_replication_causalml_amd.ops.panel import build_panel
from ate_replication_causalml_amd.reference import estimators as E

pytestmark = pytest.mark.gpu


def _close(a, b, tol):
    assert a.ate == pytest.approx(b.ate, abs=tol, rel=tol), (a, b)
    if not np.isnan(b.se):
        assert a.se == pytest.approx(b.se, abs=tol, rel=tol), (a, b)


def test_native_library_loaded(gpu):
    import os
    _native.hip()
    # ATE_DEBUG=1 (the device-assertion run) maps the debug build of the same sources
    name = "libatehip_debug.so" if os.environ.get("ATE_DEBUG", "0") not in ("", "0") \
        else "libatehip.so"
    assert any(p.endswith(name) for p in _native.loaded_libraries())


@pytest.mark.parametrize("dtype,p", [("bf16", 100), ("bf16", 150), ("bf16", 300), ("f32", 150),
                                     ("f64", 150)])
def test_gram_kernel_vs_fp64(gpu, dtype, p):
    # bf16: p=100 -> P=128 (128-tile kernel), 150 -> P=256 (one 256 tile),
    # 300 -> P=512 (256-tile kernel incl. an off-diagonal tile)
    rs = np.random.RandomState(0)
    n = 3001
    X = rs.randn(n, p) * np.linspace(0.5, 2, p) + np.linspace(-1, 1, p)
    folds = rs.randint(0, 3, n)
    pan = build_panel(X, rs.rand(n), rs.randint(0, 2, n), folds=folds, dtype=dtype, device=gpu)
    G = gram_op.gram(pan).cpu()
    ref = gram_op.gram_reference(pan)
    scale = ref.abs().max()
    tol = {"bf16": 2e-6, "f32": 2e-6, "f64": 1e-13}[dtype]
    assert ((G - ref).abs().max() / scale) < tol
    assert torch.allclose(G, G.transpose(1, 2))


@pytest.mark.parametrize("p", [400, 1000])
def test_gram_pair_kernel_vs_tile256(gpu, monkeypatch, p):
    # paired-tile (P % 512 == 0: 512, 1024 -> odd/even tile counts incl. extra off-diagonal
    # tiles) vs the three-tile 256 kernel vs fp64; symmetric by construction
    rs = np.random.RandomState(3)
    n = 6000
    X = rs.randn(n, p)
    pan = build_panel(X, rs.rand(n), rs.randint(0, 2, n), folds=rs.randint(0, 5, n),
                      dtype="bf16", device=gpu)
    monkeypatch.setattr(gram_op, "GRAM_KERNEL", "pair")
    gram_op._plan_cache.clear()
    assert gram_op.plan_for(pan).pair
    G0 = gram_op.gram(pan).clone()
    monkeypatch.setattr(gram_op, "GRAM_KERNEL", "tile256")
    gram_op._plan_cache.clear()
    G1 = gram_op.gram(pan)
    gram_op._plan_cache.clear()
    ref = gram_op.gram_reference(pan).to(gpu)
    assert ((G0 - ref).abs().max() / ref.abs().max()) < 2e-6
    assert ((G0 - G1).abs().max() / ref.abs().max()) < 2e-6
    assert torch.equal(G0, G0.transpose(1, 2))


@pytest.mark.parametrize("blocked", [False, True])
def test_gram_tri_kernel_vs_pair(gpu, monkeypatch, blocked):
    """Split-triangle kernel (P == 512, csrc/gram.hip gram_bf16_tri_kernel) vs the paired-tile
    kernel vs fp64, on a column-major and on a 64-row blocked panel; symmetric, every block
    written once (the slab table covers the triangle: tests/test_gram_plan.py)."""
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    if blocked:
        pan = synthetic_panel(40000, p=480, folds=5, seed=5, dtype="bf16", blocked=True,
                              device=gpu)
    else:
        rs = np.random.RandomState(5)
        n = 7000
        pan = build_panel(rs.randn(n, 400), rs.rand(n), rs.randint(0, 2, n),
                          folds=rs.randint(0, 5, n), dtype="bf16", device=gpu)
    assert pan.P == 512
    gram_op._plan_cache.clear()
    monkeypatch.setattr(gram_op, "GRAM_TRI", True)
    assert gram_op.plan_for(pan).tri
    Gt = gram_op.gram(pan).clone()
    gram_op._plan_cache.clear()
    monkeypatch.setattr(gram_op, "GRAM_TRI", False)
    assert not gram_op.plan_for(pan).tri
    Gp = gram_op.gram(pan).clone()
    gram_op._plan_cache.clear()
    ref = gram_op.gram_reference(pan).to(gpu)
    scale = ref.abs().max()
    assert ((Gt - ref).abs().max() / scale) < 2e-6
    assert ((Gt - Gp).abs().max() / scale) < 2e-6
    assert torch.equal(Gt, Gt.transpose(1, 2))


def test_byte_columns_gram_same_bits(gpu, monkeypatch):
    """One-byte columns (data/device_dgp.synthetic_panel: the {0, 1} columns in physical
    columns 384..511 plus a byte copy; csrc/gram.hip streams the copy as bf16 halves and the
    reduce scales back): the Gram equals the all-bf16 read BIT FOR BIT (default and exact
    mode), the byte copy holds exactly the panel's columns, and the DML-ATE is unchanged."""
    from ate_replication_causalml_amd.data import device_dgp
    from ate_replication_causalml_amd.data.device_dgp import BYTE_COL0, synthetic_panel
    from ate_replication_causalml_amd.estimators.lasso import dml_crossfit_panel
    monkeypatch.setattr(device_dgp, "BYTE_PANEL", True)
    pan = synthetic_panel(40000, p=500, folds=5, seed=5, dtype="bf16", blocked=True,
                          device=gpu, dgp="tutorial", align=4096)
    assert pan.P == 512 and pan.bytes8 is not None
    Xc = pan.colmajor()
    r = torch.arange(64, device=gpu)                 # byte position of row r (csrc/dgp.hip x8_pos)
    pos = ((r >> 3) & 3) * 16 + (r >> 5) * 8 + (r & 7)
    assert torch.equal(torch.sort(pos).values, r)
    b = pan.bytes8[:, :, pos].permute(1, 0, 2).reshape(512 - BYTE_COL0, -1)
    assert torch.equal(b, (Xc[BYTE_COL0:] != 0).to(torch.uint8) * 0x3F)
    assert torch.all((Xc[BYTE_COL0:] == 0) | (Xc[BYTE_COL0:] == 1))
    res = {}
    for on in (True, False):
        monkeypatch.setattr(gram_op, "BYTE_COLS", on)
        gram_op._plan_cache.clear()
        G = gram_op.gram(pan).clone()
        GX = gram_op.gram(pan, exact=True).clone()
        r, _, _ = dml_crossfit_panel(pan, 5)
        res[on] = (G, GX, r.cpu())
    gram_op._plan_cache.clear()
    assert torch.equal(res[True][0], res[False][0])
    assert torch.equal(res[True][1], res[False][1])
    assert torch.equal(res[True][2], res[False][2])
    ref = gram_op.gram_reference(pan).to(gpu)
    assert ((res[True][0] - ref).abs().max() / ref.abs().max()) < 2e-6


def test_byte_column_order_matches_generator_order(gpu, monkeypatch):
    """The byte panel's physical column order only relabels columns: its DML-ATE equals the
    generator-order panel's (ATE_PANEL_BYTES=0) to rounding, and every named column holds the
    same values."""
    from ate_replication_causalml_amd.data import device_dgp
    from ate_replication_causalml_amd.estimators.lasso import dml_crossfit_panel
    kw = dict(p=500, folds=5, seed=9, dtype="bf16", blocked=True, device=gpu, dgp="tutorial")
    monkeypatch.setattr(device_dgp, "BYTE_PANEL", True)
    a = device_dgp.synthetic_panel(30000, **kw)
    monkeypatch.setattr(device_dgp, "BYTE_PANEL", False)
    b = device_dgp.synthetic_panel(30000, **kw)
    assert a.bytes8 is not None and b.bytes8 is None and a.cols != b.cols
    Xa, Xb = a.colmajor(), b.colmajor()
    for nm in ("x0", "x15", "x24", "x499", "W", "Y", "W_hi", "Y_lo", "one"):
        assert torch.equal(Xa[a.cols[nm]], Xb[b.cols[nm]]), nm
    ra = dml_crossfit_panel(a, 5)[0].cpu()
    gram_op._plan_cache.clear()
    rb = dml_crossfit_panel(b, 5)[0].cpu()
    gram_op._plan_cache.clear()
    assert torch.allclose(ra, rb, rtol=1e-9, atol=1e-12), (ra, rb)


def test_invalid_launch_is_named(gpu):
    """A launch the runtime refuses (2,048 work-items per block) surfaces as NativeError
    with the HIP error's name, the entry point and the launch site (csrc/errors.hip), and
    leaves no error pending for the next op. Under ATE_DEBUG=1 the load-time resource check
    of the registered heavy kernels ran and passed."""
    import torch
    from ate_replication_causalml_amd import _native
    with pytest.raises(_native.NativeError) as ei:
        _native.call("ate_debug_bad_launch", 2048, torch.cuda.current_stream().cuda_stream)
    msg = str(ei.value)
    assert "hipError" in msg and "ate_debug_bad_launch" in msg and "errors.hip" in msg, msg
    assert ei.value.status > 0
    _native.call("ate_debug_bad_launch", 64, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    rep = _native.kernel_resource_report()
    if _native.hip_library_path().name.endswith("_debug.so"):
        assert rep and "FAIL" not in rep and "forest_exact_kernel" in rep, rep
    print(msg)


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_weighted_gram_kernel(gpu, dtype):
    rs = np.random.RandomState(1)
    X = rs.randn(1000, 20)
    pan = build_panel(X, None, rs.rand(1000), dtype=dtype, device=gpu)
    w = pan.gather_rows(torch.as_tensor(rs.rand(1000) + 0.1, device=gpu).to(pan.dtype))
    G = gram_op.gram(pan, w).cpu()
    ref = gram_op.gram_reference(pan, w)
    tol = 2e-6 if dtype == "f32" else 1e-13
    assert ((G - ref).abs().max() / ref.abs().max()) < tol


def test_chol_solve_kernel_vs_cpu(gpu):
    rs = np.random.RandomState(2)
    X = rs.randn(500, 6)
    X[:, 4] = X[:, 0] - 2 * X[:, 3]
    y = rs.randn(500)
    pan = build_panel(X, None, y, dtype="f64", device=gpu)
    G = gram_op.gram(pan)[0]
    cols = [pan.cols["one"], *pan.xcols]
    r = chol_solve(G, cols, pan.cols["Y"])
    rc = chol_solve(G.cpu(), cols, pan.cols["Y"])
    b, bc = r.beta.cpu().numpy(), rc.beta.numpy()
    assert np.array_equal(np.isnan(b), np.isnan(bc)) and np.isnan(b[5])
    assert np.allclose(np.nan_to_num(b), np.nan_to_num(bc), rtol=1e-10)
    assert np.allclose(np.nan_to_num(r.invdiag.cpu().numpy()), np.nan_to_num(rc.invdiag.numpy()),
                       rtol=1e-10)
    assert np.allclose(r.aux.cpu().numpy()[:2], rc.aux.numpy()[:2], rtol=1e-9)


def test_irls_kernel_vs_cpu(gpu):
    rs = np.random.RandomState(3)
    X = rs.randn(4000, 8)
    y = (rs.rand(4000) < 1 / (1 + np.exp(-(X[:, 0] - 0.5 * X[:, 1])))).astype(float)
    pan = build_panel(X, y, None, dtype="f64", device=gpu, extra_cols=("z",))
    cols = [pan.cols["one"], *pan.xcols]
    fit = logistic_irls(pan, cols, pan.cols["W"], pan.cols["z"])
    from ate_replication_causalml_amd.reference.linear import glm_logit
    ref = glm_logit(X, y)
    assert np.allclose(fit.beta.cpu().numpy(), ref.coef, rtol=1e-8, atol=1e-10)
    assert int(fit.state[2].item()) == ref.iters and fit.state[3].item() == 1.0
    mu = pan.scatter_rows(fit.mu).cpu().numpy()
    assert np.allclose(mu, ref.fitted, atol=1e-10)
    eta = predict(pan, cols, fit.beta, link="logit")
    assert np.allclose(pan.scatter_rows(eta).cpu().numpy(), ref.fitted, atol=1e-10)


def test_score_kernels_vs_cpu(gpu):
    rs = np.random.RandomState(4)
    n = 20000
    w = (rs.rand(n) < 0.3).astype(float)
    y = (rs.rand(n) < 0.4).astype(float)
    p = np.clip(rs.rand(n), 0.05, 0.95)
    p[:3] = [0.0, 1.0, 0.0]
    mu0, mu1 = rs.rand(n), rs.rand(n)
    t = lambda a: torch.as_tensor(a, device=gpu)
    r, m = S.naive(t(y), t(w))
    rc, mc = S.naive(torch.as_tensor(y), torch.as_tensor(w))
    assert torch.allclose(r.cpu(), rc, rtol=1e-12)
    pg = S.clip_propensity_(t(p.copy()))
    pc = E.clip_propensity(p)
    assert np.allclose(pg.cpu().numpy(), pc)
    ra, _ = S.aipw(t(w), t(y), pg, t(mu0), t(mu1))
    tau = E.aipw_point(w, y, pc, mu0, mu1)
    se = E.aipw_sandwich_se(w, y, pc, mu0, mu1, tau)
    assert np.allclose(ra.cpu().numpy(), [tau, se], rtol=1e-10)
    yr, wr = rs.randn(n), rs.randn(n)
    mg = S.dml_moments(t(yr), t(wr))
    mcpu = S.dml_moments(torch.as_tensor(yr), torch.as_tensor(wr))
    assert torch.allclose(mg.cpu(), mcpu, rtol=1e-11)
    for mode in ("plr", "lm"):
        assert torch.allclose(S.dml_finalize(mg, mode).cpu(), S.dml_finalize(mcpu, mode), rtol=1e-11)


def test_bootstrap_kernel_matches_philox_reference(gpu):
    rs = np.random.RandomState(5)
    e1 = rs.randn(3000)
    e1[7] = np.nan
    e2 = rs.randn(3000)
    tg = S.bootstrap_multinomial(torch.as_tensor(e1, device=gpu), torch.as_tensor(e2, device=gpu),
                                 64, seed=1991)
    tc = S.bootstrap_multinomial(torch.as_tensor(e1), torch.as_tensor(e2), 64, seed=1991)
    assert np.allclose(tg.cpu().numpy(), tc.numpy(), rtol=1e-11)   # same Philox draws


def test_enet_cv_kernels_vs_cpu(gpu):
    from ate_replication_causalml_amd.ops.enet import cv_enet_gaussian
    from ate_replication_causalml_amd.parallel import rng
    rs = np.random.RandomState(6)
    n, p = 3000, 70
    X = rs.randn(n, p)
    y = X[:, :4] @ [1.0, -1.0, 0.5, 0.25] + rs.randn(n)
    fid = rng.fold_ids(n, 10, 1)
    pan = build_panel(X, None, y, folds=fid, dtype="f64", device=gpu)
    G = gram_op.gram(pan)
    pf = np.ones(p)
    pf[-1] = 0
    rg = cv_enet_gaussian(G, pan, pan.xcols, [pan.cols["Y"]], penalty_factor=pf)
    rc = cv_enet_gaussian(G.cpu(), pan, pan.xcols, [pan.cols["Y"]], penalty_factor=pf)
    nl = int(rc.nlam[0])
    assert int(rg.nlam[0]) == nl
    assert np.allclose(rg.lambdas[0, :nl].cpu().numpy(), rc.lambdas[0, :nl].numpy(), rtol=1e-12)
    assert np.allclose(rg.coef_path[0, :nl].cpu().numpy(), rc.coef_path[0, :nl].numpy(),
                       atol=1e-6)
    assert torch.equal(rg.sel.cpu().long(), rc.sel.long())
    assert np.allclose(rg.cvm[0, :nl].cpu().numpy(), rc.cvm[0, :nl].numpy(), rtol=1e-6)


def test_enet_cross_lane_primitives(gpu):
    """csrc/enet.hip row_replicate (permlane32/16 swaps) and fmac_bcast (DPP64
    row_newbcast), the broadcasts of the row-blocked lasso walk, on gfx950."""
    out = torch.zeros(320, dtype=torch.float64, device=gpu)
    _native.call("ate_enet_isa_selftest", out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    o = out.cpu().numpy()
    lane = np.arange(64)
    for r in range(4):
        np.testing.assert_array_equal(o[r * 64:(r + 1) * 64], 16 * r + (lane & 15))
    np.testing.assert_array_equal(o[256:], 1 + 2 * (16 * (lane >> 4) + 5))


def test_enet_fold_wait_timeout_poisons_and_raises(gpu, monkeypatch):
    """The CV fold problems spin (bounded) on their full-data problem's lambda progress
    (csrc/enet.hip). Forcing the bound to zero polls makes fold waits time out: the launch
    must come back (no hang), flag the folds (npass < 0), NaN-poison the CV curve and the
    selection, and EnetCvResult.check() must raise; with the default bound the same call
    is clean again."""
    from ate_replication_causalml_amd.ops.enet import cv_enet_gaussian
    from ate_replication_causalml_amd.parallel import rng
    from ate_replication_causalml_amd.utils.guards import NumericalError
    rs = np.random.RandomState(7)
    n, p = 4000, 120
    X = rs.randn(n, p)
    y = X[:, :6] @ [1.0, -1.0, 0.5, 0.25, 0.2, -0.3] + rs.randn(n)
    pan = build_panel(X, None, y, folds=rng.fold_ids(n, 10, 1), dtype="f64", device=gpu)
    G = gram_op.gram(pan)
    monkeypatch.setenv("ATE_ENET_SPIN_MAX", "0")
    r = cv_enet_gaussian(G, pan, pan.xcols, [pan.cols["Y"]])
    torch.cuda.synchronize()
    bad = (r.fold_npass < 0).cpu().numpy()
    assert bad.any(), "no fold wait timed out with a zero spin bound"
    assert torch.isnan(r.cvm).all() and torch.isnan(r.coef_min).all()
    with pytest.raises(NumericalError):
        r.check()
    monkeypatch.delenv("ATE_ENET_SPIN_MAX")
    ok = cv_enet_gaussian(G, pan, pan.xcols, [pan.cols["Y"]]).check()
    assert (ok.fold_npass >= 0).all() and torch.isfinite(ok.coef_min).all()


def test_device_estimators_vs_reference(gpu, tutorial):
    from ate_replication_causalml_amd.estimators import lasso as DL
    from ate_replication_causalml_amd.estimators import linear as D
    _, m, _ = tutorial
    Y, W, X = m.Y, m.W, m.X
    _close(D.naive(Y, W, device=gpu), E.naive(Y, W), 1e-12)
    _close(D.ols(Y, W, X, device=gpu), E.ols(Y, W, X), 1e-9)
    p = E.propensity_logistic(W, X)
    assert np.abs(D.propensity_logistic(W, X, device=gpu).cpu().numpy() - p).max() < 1e-9
    for compat in ("reference", "textbook"):
        _close(D.ipw(Y, W, X, p, compat=compat, device=gpu), E.ipw(Y, W, X, p, compat=compat), 1e-8)
    _close(D.ipw_wls(Y, W, p, device=gpu), E.ipw_wls(Y, W, p), 1e-9)
    _close(D.aipw_glm(Y, W, X, device=gpu), E.aipw_glm(Y, W, X), 1e-8)
    _close(D.aipw_glm(Y, W, X, bootstrap_se=True, B=100, device=gpu),
           E.aipw_glm(Y, W, X, bootstrap_se=True, B=100), 1e-8)
    _close(DL.lasso_single(Y, W, X, device=gpu), E.lasso_single(Y, W, X), 1e-6)
    _close(DL.lasso_usual(Y, W, X, device=gpu), E.lasso_usual(Y, W, X), 1e-6)
    _close(DL.dml_plr_lasso(Y, W, X, device=gpu), E.dml_plr_lasso(Y, W, X), 1e-6)


def test_belloni_gpu_vs_reference(gpu, tutorial):
    from ate_replication_causalml_amd.estimators import lasso as DL
    _, m, _ = tutorial
    a = DL.belloni(m.Y, m.W, m.X, device=gpu)
    b = E.belloni(m.Y, m.W, m.X)
    _close(a, b, 1e-6)


def test_device_dgp_matches_host(gpu):
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    pg = synthetic_panel(5000, p=30, folds=5, seed=9, dtype="f32", device=gpu)
    pc = synthetic_panel(5000, p=30, folds=5, seed=9, dtype="f64", device="cpu")
    a = pg.data[:pc.P].double().cpu()[:, : pc.ld]
    b = pc.data[:, : pg.ld]
    assert pg.ld == pc.ld
    diff = (a[: b.shape[0]] - b).abs()
    # continuous columns agree to fp32 Box-Muller accuracy; binary thresholds may flip
    # on a handful of draws sitting exactly at the threshold
    assert (diff > 1e-3).float().mean() < 1e-4


def test_dml_bf16_vs_f64_panel(gpu):
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.lasso import dml_crossfit_panel
    pb = synthetic_panel(200000, p=60, folds=5, seed=2, dtype="bf16", device=gpu)
    p64 = synthetic_panel(200000, p=60, folds=5, seed=2, dtype="f64", device=gpu)
    rb, _, _ = dml_crossfit_panel(pb, 5)
    r64, _, _ = dml_crossfit_panel(p64, 5)
    rb, r64 = rb.cpu().numpy(), r64.cpu().numpy()
    # bf16 storage quantises the continuous covariates (rel 2^-9); the ATE moves by far
    # less than its standard error
    assert abs(rb[0] - r64[0]) < 0.05 * r64[1]
    assert abs(rb[1] - r64[1]) < 0.02 * r64[1]


def test_smoke_entry(gpu):
    import __graft_entry__
    __graft_entry__.smoke()


def test_dml_two_graphs_in_flight_match_eager(gpu):
    """bench.py --inflight: two captured cross-fits with private Gram workspaces
    (ops/gram.plan_slot) replayed concurrently on two streams give the eager result."""
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.lasso import dml_crossfit_panel
    from ate_replication_causalml_amd.utils.graphs import GraphedStep
    pan = synthetic_panel(100000, p=500, folds=5, seed=4, dtype="bf16", device=gpu)

    def step():
        return dml_crossfit_panel(pan, 5, "min")[0]

    want = step().clone()
    runs = []
    for i in range(2):
        with gram_op.plan_slot(i):
            runs.append(GraphedStep(step))
    streams = [torch.cuda.Stream(gpu) for _ in runs]
    assert runs[0].out.data_ptr() != runs[1].out.data_ptr()
    for k in range(6):
        with torch.cuda.stream(streams[k % 2]):
            runs[k % 2]()
    torch.cuda.synchronize()
    for r in runs:
        torch.testing.assert_close(r.out, want, rtol=0, atol=0)


def test_spd_solve_batched_vs_fp64_reference(gpu):
    """csrc/linalg.hip spd_solve_kernel (the balancing QP's Schur solves, capturable) against
    torch.linalg.solve in fp64 on the host; a non-SPD system comes back NaN."""
    import torch
    from ate_replication_causalml_amd.ops.linalg import spd_solve
    g = torch.Generator().manual_seed(5)
    A, k = 3, 43
    M = torch.randn(A, k, k, generator=g, dtype=torch.float64)
    K = M @ M.transpose(1, 2) + k * torch.eye(k, dtype=torch.float64)
    K[2] = -K[2]                                   # not positive definite
    r = torch.randn(A, k, generator=g, dtype=torch.float64)
    x = spd_solve(K.to(gpu), r.to(gpu)).cpu()
    want = torch.linalg.solve(K[:2], r[:2, :, None])[:, :, 0]
    assert torch.allclose(x[:2], want, rtol=1e-12, atol=1e-14)
    assert torch.isnan(x[2]).all()


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_weighted_gram_bitwise_repeatable(gpu, dtype):
    """Row-weighted Gram (IRLS / WLS / balancing steps): every entry has one writer in the
    slab reduce, so repeated calls are bit-identical (two writers per diagonal-tile entry
    made it differ at rounding level) and the result is exactly symmetric."""
    import torch
    from ate_replication_causalml_amd.ops.gram import gram
    from ate_replication_causalml_amd.ops.panel import build_panel
    rs = np.random.RandomState(4)
    X = rs.randn(3000, 9)
    pan = build_panel(X, None, rs.randn(3000), folds=rs.randint(0, 4, 3000), dtype=dtype,
                      device=gpu)
    w = torch.as_tensor(rs.rand(pan.ld), device=gpu).to(pan.data.dtype)
    Gs = [gram(pan, w=w).clone() for _ in range(3)]
    assert all(torch.equal(Gs[0], g) for g in Gs[1:])
    assert torch.equal(Gs[0], Gs[0].transpose(1, 2))


def test_bench_eager_gram_matches_graph_gram(gpu):
    """bench.py's in-flight block: the Gram as a plain launch on the Gram stream (the
    default, ATE_BENCH_EAGER_GRAM=1) and as a one-node graph give the same ATE/SE bits, the
    in-flight fits agree with each other and with the timed single call. The repeated
    cross-fitting block (3 partitions of 25 micro-segments, one graph) reports 3 distinct
    split ATEs whose median is the aggregate, and partition 0 (micro-segment m -> fold
    m // 5: the main panel's folds) matches the single call up to Gram chunking."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for eg in ("0", "1"):
        env = dict(os.environ, ATE_BENCH_EAGER_GRAM=eg)
        r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--rows", "1e6",
                            "--steps", "2", "--warmup", "1", "--parity", "0", "--also-rct", "0"],
                           capture_output=True, text=True, env=env, timeout=200)
        assert r.returncode == 0, r.stderr[-2000:]
        line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
        d = json.loads(line)
        inf = d["throughput_inflight"]
        assert inf["inflight"] == 3 and inf["stagger"]
        assert inf["fits_agree"]                   # the three in-flight fits: same bits
        # another Gram chunking than the single call: equal up to fp32 partial-sum rounding
        assert inf["abs_diff_ate_vs_single"] <= 1e-3 * d["se"]
        assert inf["rel_diff_se_vs_single"] <= 1e-4
        out[eg] = (inf["ate_hex"], inf["se_hex"])
        rep = d["repeated"]
        assert rep["repeats"] == 3 and rep["hipgraph"] and rep["splits_distinct"]
        a = sorted(s[0] for s in rep["splits"])
        assert rep["ate"] == a[1]
        assert abs(rep["splits"][0][0] - d["ate"]) <= 1e-3 * d["se"]
    assert out["0"] == out["1"]


def test_repeated_dml_gpu_matches_host_and_graph(gpu):
    """Repeated cross-fitting (3 partitions from one 25-segment Gram pass) on the GPU: equal
    to the host run of the same device pipeline, and its captured-graph replays (2nd and
    3rd call) equal the eager first call."""
    from ate_replication_causalml_amd.estimators import lasso as L
    rs = np.random.RandomState(8)
    n, p = 6000, 30
    X = rs.randn(n, p)
    W = (rs.rand(n) < 1 / (1 + np.exp(-X[:, 0]))).astype(float)
    Y = X[:, 1] + 0.5 * W + rs.randn(n)
    c = L.dml_plr_lasso_repeated(Y, W, X, 5, 3, device="cpu")
    outs = [L.dml_plr_lasso_repeated(Y, W, X, 5, 3, device=gpu) for _ in range(3)]
    assert [o.diagnostics["hipgraph"] for o in outs] == [False, True, True]
    for o in outs:
        assert o.ate == pytest.approx(c.ate, rel=1e-9) and o.se == pytest.approx(c.se, rel=1e-9)
        np.testing.assert_allclose(o.diagnostics["splits"], c.diagnostics["splits"], rtol=1e-9)
    assert outs[1].ate == outs[0].ate and outs[2].se == outs[0].se
