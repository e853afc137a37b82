"""GPU forest kernels (csrc/forest.hip) against the host C++ engine: every split
statistic is an integer or 2^-32 fixed-point sum and both sides draw from the same
Philox streams, so the trees must be bit-identical, not merely close."""
import numpy as np
import pytest

from ate_replication_causalml_amd.models import forest as F

from test_forest import _toy, assert_same_forest

pytestmark = pytest.mark.gpu


def _np(a):
    return a.cpu().numpy() if hasattr(a, "cpu") else np.asarray(a)


def _data(n=3000):
    X = _toy(n=n, p=8, seed=3)
    r = np.random.default_rng(4)
    W = (r.uniform(size=n) < 1 / (1 + np.exp(-X[:, 2]))).astype(float)
    Y = X[:, 1] + (1 + (X[:, 0] > 0)) * W + 0.5 * r.normal(size=n)
    return X, W, Y


def test_bin_matrix_gpu_matches_host(gpu):
    X, _, _ = _data()
    edges, ne = F.bin_edges(X)
    a = F.bin_matrix(X, edges, ne, gpu).cpu().numpy()
    b = F.bin_matrix(X, edges, ne, None).numpy()
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("nw", ["0", "4", "8", "16"])
@pytest.mark.parametrize("case", ["rf_class", "rf_reg", "grf_reg", "causal"])
def test_forest_gpu_bit_identical_to_host(gpu, case, nw, monkeypatch):
    """Every instantiation of the grow kernel (waves per tree 4 / 8 / 16 with their
    register budgets, and the automatic choice) grows the host engine's trees."""
    monkeypatch.setenv("ATE_FOREST_NW", nw)
    X, W, Y = _data()
    kw = dict(ntree=24, seed=17)
    if case == "rf_class":
        kw.update(kind=F.KIND_CLASS, y=W, mtry=3)
    elif case == "rf_reg":
        kw.update(kind=F.KIND_REG, r1=Y, mtry=3, min_node=5)
    else:
        kw.update(mtry=F.grf_mtry(8), min_node=5, sampling=1, honesty=True, group=2,
                  mtry_poisson=True, alpha=0.05, sample_fraction=0.5)
        if case == "grf_reg":
            kw.update(kind=F.KIND_REG, r1=Y)
        else:
            kw.update(kind=F.KIND_CAUSAL, r1=W - W.mean(), r2=Y - Y.mean())
    g = F.fit_forest(X, backend="gpu", **kw)
    c = F.fit_forest(X, backend="cpu", **kw)
    assert_same_forest(g, c)
    if g.est is not None:
        # honest estimation-sample sufficient statistics of every node
        nn = _np(g.nnodes)
        ge, ce = _np(g.est).reshape(kw["ntree"], -1, 5), _np(c.est).reshape(kw["ntree"], -1, 5)
        for t in range(kw["ntree"]):
            np.testing.assert_array_equal(ge[t, :nn[t]], ce[t, :nn[t]])
    for oob in (True, False):
        pg = g.predict_raw(None if oob else X[:500], oob=oob)
        pc = c.predict_raw(None if oob else X[:500], oob=oob)
        np.testing.assert_allclose(pg, pc, rtol=1e-12, atol=1e-12, equal_nan=True)


def test_device_forest_estimators_match_host(gpu, tutorial):
    from ate_replication_causalml_amd.estimators import forest as DF
    _, m, _ = tutorial
    Y, W, X = m.Y, m.W, m.X
    for f in (lambda d: DF.aipw_rf(Y, W, X, num_trees=60, device=d),
              lambda d: DF.double_ml(Y, W, X, num_trees=40, device=d),
              lambda d: DF.causal_forest_ate(Y, W, X, num_trees=80, device=d, compat="textbook"),
              # the default (compat="reference", W.hat unclipped; here in [0.07, 0.26])
              lambda d: DF.causal_forest_ate(Y, W, X, num_trees=80, device=d)):
        a, b = f(gpu), f("cpu")
        assert np.isfinite(a.ate) and np.isfinite(a.se)
        assert a.ate == pytest.approx(b.ate, rel=1e-9, abs=1e-12)
        assert a.se == pytest.approx(b.se, rel=1e-9, abs=1e-12)
        for k in ("w_hat_min", "w_hat_max"):
            if k in a.diagnostics:
                assert a.diagnostics[k] == pytest.approx(b.diagnostics[k], rel=1e-12)


def test_causal_forest_default_compat_overlap(gpu, tutorial):
    """compat="reference" (grf: W.hat not clipped). The tutorial df_mod keeps W.hat inside
    (0, 1): the bootstrap SE path agrees with the host. Tiny orthogonalisation forests (12
    trees) on the toy data leave W.hat at exactly 0 for some rows: then the AIPW scores are
    infinite on both devices, as in grf, and the overlap warning fires on both."""
    import warnings
    from ate_replication_causalml_amd.estimators import crossfit as CF
    _, m, _ = tutorial
    a = CF.causal_forest_bootstrap(m.Y, m.W, m.X, num_trees=24, B=64, device=gpu)
    b = CF.causal_forest_bootstrap(m.Y, m.W, m.X, num_trees=24, B=64, device="cpu")
    assert np.isfinite(a.ate) and np.isfinite(a.se) and a.se > 0
    assert a.ate == pytest.approx(b.ate, rel=1e-9) and a.se == pytest.approx(b.se, rel=1e-8)
    X, W, Y = _data(2000)
    for dev in (gpu, "cpu"):
        with warnings.catch_warnings(record=True) as ws:
            warnings.simplefilter("always")
            r = CF.causal_forest_bootstrap(Y, W, X, num_trees=24, nuisance_trees=12, B=64,
                                           device=dev)
        assert any("poor overlap" in str(w.message) for w in ws), dev
        assert not np.isfinite(r.ate), (dev, r)


def test_crossfit_and_cf_bootstrap_gpu_match_host(gpu):
    from ate_replication_causalml_amd.estimators import crossfit as CF
    X, W, Y = _data(2000)
    Yb = (Y > np.median(Y)).astype(float)
    a = CF.aipw_crossfit(Yb, W, X, learner="rf", num_trees=20, device=gpu)
    b = CF.aipw_crossfit(Yb, W, X, learner="rf", num_trees=20, device="cpu")
    assert a.ate == pytest.approx(b.ate, rel=1e-10) and a.se == pytest.approx(b.se, rel=1e-10)
    assert a.diagnostics["device_scores"]        # nuisances + score stayed on the GPU
    for learner in ("glm", "gbdt"):
        g = CF.aipw_crossfit(Yb, W, X, learner=learner, device=gpu, gbdt_kw={"n_trees": 8})
        h = CF.aipw_crossfit(Yb, W, X, learner=learner, device="cpu", gbdt_kw={"n_trees": 8})
        assert g.ate == pytest.approx(h.ate, abs=5e-3) and g.se == pytest.approx(h.se, rel=0.05)
    c = CF.causal_forest_bootstrap(Y, W, X, num_trees=24, nuisance_trees=12, B=64, compat="textbook", device=gpu)
    d = CF.causal_forest_bootstrap(Y, W, X, num_trees=24, nuisance_trees=12, B=64, compat="textbook", device="cpu")
    assert c.ate == pytest.approx(d.ate, rel=1e-9) and c.se == pytest.approx(d.se, rel=1e-8)


def test_aipw_rf_crossfit_panel_matches_host_engine(gpu):
    """Config 3 on an HBM panel: device binning, device-gathered training columns, GPU
    forests; the host forest engine on the same bins grows the same trees (same ATE)."""
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.crossfit import aipw_rf_crossfit_panel
    pan = synthetic_panel(6000, p=30, folds=5, seed=5, dtype="bf16", device=gpu)
    a = aipw_rf_crossfit_panel(pan, num_trees=24, seed=3)
    b = aipw_rf_crossfit_panel(pan, num_trees=24, seed=3, engine="cpu")
    assert abs(a.ate - b.ate) < 1e-12 and abs(a.se - b.se) < 1e-12, (a, b)
    assert 0 < a.se < 0.1 and abs(a.ate) < 0.5
    # a tree shard of the same forests (rank 1 of 3) is a different, smaller ensemble
    c = aipw_rf_crossfit_panel(pan, num_trees=24, seed=3, tree_shard=(1, 3))
    assert c.diagnostics["trees_this_device"] == 8


@pytest.mark.parametrize("layout", ["row", "col"])
@pytest.mark.parametrize("big,chunk", [(65536, 4096), (8192, 4096), (300, 128), (65, 64)])
@pytest.mark.parametrize("case", ["rf_class", "rf_reg"])
def test_level_engine_bit_identical_to_host(gpu, case, big, chunk, layout, monkeypatch):
    """The level-synchronous engine (csrc/forest_level.hip: all trees level by level, big
    nodes over many workgroups, mid nodes a workgroup, small nodes a wave) grows the host
    engine's trees bit for bit. Small thresholds push most nodes through the big /
    chunked-partition paths (every node class and both partition paths are exercised);
    both layouts of the growth copy (row-major, column-major)."""
    monkeypatch.setenv("ATE_FOREST_ENGINE", "level")
    monkeypatch.setenv("ATE_FOREST_LV_BIG", str(big))
    monkeypatch.setenv("ATE_FOREST_LV_CH", str(chunk))
    monkeypatch.setenv("ATE_FOREST_LV_ITEMS", "100000")   # keep the small chunks
    monkeypatch.setenv("ATE_FOREST_LV_T2", str(max(65, big // 2)))
    monkeypatch.setenv("ATE_FOREST_LV_LAYOUT", layout)
    X, W, Y = _data(6000)
    kw = dict(ntree=12, seed=23)
    if case == "rf_class":
        kw.update(kind=F.KIND_CLASS, y=W, mtry=3)
    else:
        kw.update(kind=F.KIND_REG, r1=Y, mtry=3, min_node=5)
    g = F.fit_forest(X, backend="gpu", **kw)
    c = F.fit_forest(X, backend="cpu", **kw)
    assert_same_forest(g, c)
    np.testing.assert_array_equal(_np(g.inbag), _np(c.inbag))
    np.testing.assert_array_equal(g.oob_proba(), c.oob_proba())


def test_level_engine_wide_many_features(gpu, monkeypatch):
    """p = 120, mtry = 10 (two feature groups per histogram pass), trees with > 60 levels
    of nodes: same trees as the per-tree kernel."""
    monkeypatch.setenv("ATE_FOREST_LV_BIG", "512")
    monkeypatch.setenv("ATE_FOREST_LV_CH", "256")
    r = np.random.default_rng(8)
    n, p = 20000, 120
    X = r.normal(size=(n, p))
    X[:, 5] = np.round(X[:, 5])
    W = (r.uniform(size=n) < 1 / (1 + np.exp(-X[:, 0] - X[:, 7] * X[:, 9]))).astype(float)
    kw = dict(kind=F.KIND_CLASS, y=W, ntree=6, seed=5, mtry=10)
    monkeypatch.setenv("ATE_FOREST_ENGINE", "level")
    g = F.fit_forest(X, backend="gpu", **kw)
    monkeypatch.setenv("ATE_FOREST_ENGINE", "tree")
    t = F.fit_forest(X, backend="gpu", **kw)
    assert_same_forest(g, t)


@pytest.mark.parametrize("n", [3000, 7000, 20000, 40000])
@pytest.mark.parametrize("case", ["rf_class", "rf_reg"])
def test_exact_split_engine_bit_identical_to_host(gpu, case, n):
    """csrc/forest_exact.hip (sort-based splits on uint16 value ranks: lane-per-row nodes
    <= 64 rows, wave bitonic sorts in LDS <= 256 rows (EXACT_WCAP), workgroup bitonic sorts
    in LDS <= 8192 rows (EXACT_XLDS) -- the n = 3000 / 7000 roots -- and in global scratch
    above -- n = 20000 / 40000) grows the host twin's trees bit for bit; OOB and new-row
    predictions match."""
    r = np.random.default_rng(11)
    X = r.normal(size=(n, 7))
    X[:, 3] = np.round(X[:, 3])                 # a few ties / repeated values
    W = (r.uniform(size=n) < 1 / (1 + np.exp(-X[:, 0] - X[:, 1] * X[:, 2]))).astype(float)
    Y = X[:, 1] + W * (1 + X[:, 0]) + 0.5 * r.normal(size=n)
    kw = dict(ntree=10, seed=13, splits="exact")
    if case == "rf_class":
        kw.update(kind=F.KIND_CLASS, y=W)
    else:
        kw.update(kind=F.KIND_REG, r1=Y, min_node=5, mtry=3)
    g = F.fit_forest(X, backend="gpu", **kw)
    c = F.fit_forest(X, backend="cpu", **kw)
    assert_same_forest(g, c)
    np.testing.assert_array_equal(g.oob_proba(), c.oob_proba())
    np.testing.assert_array_equal(g.predict_proba(X[:700]), c.predict_proba(X[:700]))


@pytest.mark.parametrize("n", [3000, 20000])
@pytest.mark.parametrize("case", ["grf_reg_g1", "grf_reg_g2", "grf_causal"])
def test_exact_grf_engine_bit_identical_to_host(gpu, case, n):
    """grf semantics on the exact-split engine: half-samples / little bags
    (group 2) or direct subsamples (group 1, grf's orthogonalisation forests), honesty with
    the J2 estimation statistics, kind-2 causal splits on pseudo-outcomes with the
    treated / control constraint, the left value as threshold -- csrc/forest_exact.hip grows
    the host twin's trees and estimation statistics bit for bit; OOB predictions (honest
    leaves, little-bag variance) match."""
    r = np.random.default_rng(12)
    X = r.normal(size=(n, 6))
    X[:, 2] = np.round(X[:, 2] * 2)             # ties
    W = (r.uniform(size=n) < 1 / (1 + np.exp(-X[:, 0]))).astype(float)
    Y = X[:, 1] + W * (1 + (X[:, 0] > 0)) + 0.5 * r.normal(size=n)
    grf = dict(ntree=8, seed=21, splits="exact", sampling=1, honesty=True, mtry_poisson=True,
               min_node=5, alpha=0.05, sample_fraction=0.5, mtry=F.grf_mtry(6))
    if case == "grf_reg_g1":
        grf.update(kind=F.KIND_REG, r1=Y, group=1)
    elif case == "grf_reg_g2":
        grf.update(kind=F.KIND_REG, r1=W, group=2)
    else:
        grf.update(kind=F.KIND_CAUSAL, r1=W - W.mean(), r2=Y - Y.mean(), group=2)
    g = F.fit_forest(X, backend="gpu", **grf)
    c = F.fit_forest(X, backend="cpu", **grf)
    assert_same_forest(g, c)
    np.testing.assert_array_equal(g.est.cpu().numpy(), np.asarray(c.est))
    np.testing.assert_array_equal(g.predict_raw(None, oob=True), c.predict_raw(None, oob=True))
