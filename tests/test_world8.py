"""World 8 -- the whole target node (BASELINE configs 3-5: 8 x MI355X) -- rehearsed on the
CPU for every sharded path ("bitwise-identical ... across world sizes
1/2/4/8"). The thread simulator (parallel/comm.run_simulated: ranks = threads, the
collectives of the real communicator in a fixed order) runs each path at world 8 against
world 1, plus one real ``torch.distributed.run --nproc-per-node=8`` (gloo) run of bench.py.
Integer / exact paths are compared with rtol = 0.

Edge cases that only appear at 8 ranks and are pinned here:
* more ranks than outer folds: in the DML step, ranks 5-7 solve no CV paths (the path
  solves are sharded by outer fold, estimators/lasso.dml_phases) and contribute zeros;
* C04 with 8 feature slices (models/gbdt.c04_slices(40, 8) = 8 x 5 columns);
* config 4's little bags and bootstrap replicates split 8 ways, neither a multiple of 8;
* the selection transform's candidate blocks counted over 8 shares (plan_selection).
Reference ancestors: /root/reference/ate_functions.R:188-195 (the replicate loop sharded
here), :169-174 / :340-349 (the forests sharded by tree), :101-103 (cv.glmnet)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from ate_replication_causalml_amd.data import dgp
from ate_replication_causalml_amd.data.device_dgp import fold_slices, synthetic_panel
from ate_replication_causalml_amd.data.panel_selection import kept_gids, plan_selection
from ate_replication_causalml_amd.estimators import crossfit as CF
from ate_replication_causalml_amd.estimators.lasso import dml_crossfit_panel
from ate_replication_causalml_amd.parallel.comm import LocalComm, run_simulated
from ate_replication_causalml_amd.parallel.dist import DistContext

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W8 = 8


def test_dml_exact_world8_bitwise_and_idle_path_ranks():
    """Exact-mode DML (block-aligned shards, int64-limb Gram all-reduce, exact moments) at
    world 8 = world 1 bit for bit. 5 outer folds over 8 ranks: ranks 5, 6, 7 run no path
    solve (their coefficient rows are zeros before C08)."""
    from ate_replication_causalml_amd.estimators import lasso as L
    n, p, blk = 4000, 24, 64

    def run(world, rank, comm):
        pan = synthetic_panel(n, p=p, folds=5, seed=3, dtype="f64", device="cpu", rank=rank,
                              world=world, align=blk)
        res, mom, cv = dml_crossfit_panel(pan, 5, comm=comm, exact=True)
        return res.numpy(), mom.numpy(), cv is not None
    ref, mref, _ = run(1, 0, LocalComm())
    outs = run_simulated(W8, lambda c: run(W8, c.rank, c))
    for r, (res, mom, solved) in enumerate(outs):
        np.testing.assert_array_equal(res, ref)
        np.testing.assert_array_equal(mom, mref)
        assert solved == (r < 5), (r, solved)
    # every rank held rows of every fold (8 x 64-row blocks per 800-row fold)
    for r in range(W8):
        assert all(c > 0 for _, c in fold_slices(n, 5, r, W8, blk))
    assert L.EXACT_BLOCK % blk == 0


def test_dml_default_mode_world8():
    """The default (non-exact) DML step at world 8: fp64 all-reduced sufficient statistics,
    equal to world 1 up to summation order."""
    def run(world, rank, comm):
        pan = synthetic_panel(2400, p=24, folds=5, seed=3, dtype="f64", device="cpu",
                              rank=rank, world=world)
        return dml_crossfit_panel(pan, 5, comm=comm)[0].numpy()
    ref = run(1, 0, LocalComm())
    for res in run_simulated(W8, lambda c: run(W8, c.rank, c)):
        np.testing.assert_allclose(res, ref, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("n_keep,seed", [(6000, 7), (20000, 21)])
def test_selection_kept_set_world8(n_keep, seed):
    """The tutorial selection transform planned over 8 shares (each rank counts its
    candidate blocks, one all-reduce): the same n_gen and thresholds on every rank, and the
    kept-row sets of the 8 rank slices reassemble the world-1 kept set exactly."""
    ref_sel = plan_selection(n_keep, seed, dgp.TUTORIAL)
    ref = kept_gids(ref_sel, [(0, n_keep)]).numpy()

    def rank_rows(comm):
        sel = plan_selection(n_keep, seed, dgp.TUTORIAL, comm=comm)
        sl = fold_slices(n_keep, 5, comm.rank, comm.world_size)
        return sel, sl, kept_gids(sel, sl).numpy()
    got = np.full(n_keep, -1, dtype=np.int64)
    for sel, sl, g in run_simulated(W8, rank_rows):
        assert (sel.n_gen, sel.thr_t, sel.thr_c) == (ref_sel.n_gen, ref_sel.thr_t, ref_sel.thr_c)
        for f in ("blk_ct", "blk_cc", "blk_kept"):
            np.testing.assert_array_equal(getattr(sel, f), getattr(ref_sel, f))
        o = 0
        for a, c in sl:
            got[a:a + c] = g[o:o + c]
            o += c
    np.testing.assert_array_equal(got, ref)


def test_config3_rf_crossfit_world8_bitwise():
    """Config 3 (tools/cfg3.py's estimator) on a tutorial panel: the 15 forests' trees
    sharded 8 ways (20 trees: 3 or 2 per rank), local held-out vote sums packed and
    all-reduced once (C05, integers) -> the same ATE / SE bits as one process."""
    pan = synthetic_panel(3000, p=24, folds=5, seed=5, dtype="f32", device="cpu",
                          dgp="tutorial")
    one = CF.aipw_rf_crossfit_panel(pan, num_trees=20, seed=3)
    outs = run_simulated(W8, lambda c: CF.aipw_rf_crossfit_panel(pan, num_trees=20, seed=3,
                                                                 comm=c))
    counts = sorted(r.diagnostics["trees_this_device"] for r in outs)
    assert sum(counts) == 20 and counts[0] == 2 and counts[-1] == 3
    for r in outs:
        assert r.ate == one.ate and r.se == one.se


def test_config4_causal_forest_bootstrap_world8_bitwise():
    """Config 4 (tools/cfg4.py's estimator): causal-forest little bags sharded 8 ways (44
    trees = 22 bags of 2: 2 or 3 bags per rank), int64 fixed-point C05 sums, and 203
    bootstrap replicates split 8 ways (C07 all-gather) -> the ATE and bootstrap SE are the
    same bits as one process."""
    r = np.random.default_rng(4)
    n = 900
    X = r.normal(size=(n, 6))
    W = (r.uniform(size=n) < 0.4).astype(float)
    Y = X[:, 0] + (1 + (X[:, 1] > 0)) * W + 0.3 * r.normal(size=n)
    kw = dict(num_trees=44, nuisance_trees=12, B=203, compat="textbook", device="cpu",
              boot_chunk=25)
    one = CF.causal_forest_bootstrap(Y, W, X, **kw)
    for b in run_simulated(W8, lambda c: CF.causal_forest_bootstrap(Y, W, X, comm=c, **kw)):
        assert b.ate == one.ate and b.se == one.se


def test_config5_gbdt_world8_c04_slices_bitwise():
    """Config 5's algorithm (tools/cfg5.py: row-sharded DML-GBDT) at world 8 on 4,000 kept
    rows of the tutorial panel with p = 40: C04 reduce-scatters each level's int64
    histograms into 8 feature slices of 5 and all-gathers the split candidates; the global
    edge sample, exact base and exact moments make the ATE / SE the same bits as one
    process. (The HBM-panel twin, dml_plr_gbdt_panel, needs a GPU: it is the same C04
    scheme, pinned at 2-3 ranks by tests/test_gpu_multirank.py.)"""
    from ate_replication_causalml_amd.estimators.boosting import dml_plr_gbdt
    from ate_replication_causalml_amd.models import gbdt as G
    n, p = 4000, 40
    pan = synthetic_panel(n, p=p, folds=1, seed=8, dtype="f64", device="cpu", dgp="tutorial")
    Xc = pan.colmajor()[:, :pan.n].numpy()
    X = Xc[pan.xcols].T.copy()
    Y, W = Xc[pan.cols["Y"]].copy(), Xc[pan.cols["W"]].copy()
    kw = dict(n_trees=4, depth=3, device="cpu")
    one = dml_plr_gbdt(Y, W, X, **kw)
    calls = []
    orig = G.SlicedC04.scatter

    def spy(self, hist):
        calls.append(self.pl)
        return orig(self, hist)
    G.SlicedC04.scatter = spy
    try:
        def fn(comm):
            d = DistContext.for_rank(comm, n)
            return dml_plr_gbdt(d.local(Y), d.local(W), d.local(X), dist=d, **kw)
        outs = run_simulated(W8, fn)
    finally:
        G.SlicedC04.scatter = orig
    assert calls and set(calls) == {5}
    for r in outs:
        assert r.ate == one.ate and r.se == one.se


def test_bench_exact_gloo_world8_bitwise():
    """bench.py as the driver launches it at N = 8 (torch.distributed.run, 8 gloo ranks on
    the CPU, exact mode, tutorial panel, weak scaling) prints ONE JSON line whose ATE / SE
    bits equal one process holding all 8 ranks' kept rows (the same selection plan: same
    n_generated). 16384-row exact blocks: 82,000 rows per rank -> 8 blocks per fold."""
    bench = os.path.join(ROOT, "bench.py")
    args = ["--p", "24", "--dtype", "f64", "--exact", "1", "--steps", "1", "--warmup", "0",
            "--parity", "0", "--also-rct", "0"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        f"--nproc-per-node={W8}", "--master-addr=127.0.0.1",
                        "--master-port=29711", bench, "--gpus", str(W8), "--rows", "82000",
                        *args], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    eight = json.loads(lines[0])
    one = subprocess.run([sys.executable, bench, "--rows", str(82000 * W8), *args],
                         capture_output=True, text=True, env=env, timeout=600)
    assert one.returncode == 0, one.stderr[-3000:]
    ref = json.loads([l for l in one.stdout.splitlines() if l.startswith("{")][-1])
    assert eight["n_gpus"] == W8 and eight["config"]["parallelism"] == f"dp{W8}"
    assert eight["config"]["global_batch"] == ref["config"]["global_batch"] == 82000 * W8
    assert eight["config"]["n_generated"] == ref["config"]["n_generated"]
    assert eight["exact"] and ref["exact"]
    assert eight["ate_hex"] == ref["ate_hex"] and eight["se_hex"] == ref["se_hex"]
