"""The forest engines against an independent numpy oracle (reference/forest.py): trees grown
node by node from the written spec (csrc/forest_common.hpp header), sharing nothing with
csrc/cpu/forest_cpu.cpp or the gfx950 kernels but the Philox streams and the fixed-point
statistics. Same trees (feature, threshold bin, children, leaf values), the same in-bag
rows and the same honest estimation sums, for randomForest classification / regression and
grf regression / causal forests (little bags, honesty, Poisson mtry, alpha)."""
import numpy as np
import pytest

from ate_replication_causalml_amd.models import forest as F
from ate_replication_causalml_amd.reference import forest as R


def _data(n=160, p=6, seed=3):
    r = np.random.default_rng(seed)
    X = r.normal(size=(n, p))
    X[:, 2] = np.round(X[:, 2])                     # a few distinct values (ties in bins)
    w = (r.uniform(size=n) < 1 / (1 + np.exp(-X[:, 0]))).astype(float)
    y = X[:, 1] + 0.8 * w * (X[:, 3] > 0) + 0.3 * r.normal(size=n)
    return X, w, y


CASES = {
    "rf_class": dict(kind=0, mtry=2, min_node=1),
    "rf_reg": dict(kind=1, mtry=3, min_node=5),
    "grf_reg": dict(kind=1, sampling=1, mtry=4, min_node=5, honesty=True, group=2,
                    mtry_poisson=True, alpha=0.05),
    "grf_causal": dict(kind=2, sampling=1, mtry=4, min_node=5, honesty=True, group=2,
                       mtry_poisson=True, alpha=0.05),
    "grf_causal_g1": dict(kind=2, sampling=1, mtry=3, min_node=3, honesty=True, group=1,
                          mtry_poisson=True, alpha=0.05, sample_fraction=0.6),
    # mtry > 8: the exact engine's list-only instantiation (csrc/forest_exact.hip SMALL_MTRY)
    "grf_causal_m12": dict(kind=2, sampling=1, mtry=12, min_node=5, honesty=True, group=2,
                           mtry_poisson=True, alpha=0.05, p=14),
    "rf_reg_m10": dict(kind=1, mtry=10, min_node=5, p=14),
}


def _fit_both(name, backend="cpu", ntree=4, t0=0, exact=False, n=160):
    c = CASES[name]
    X, w, y = _data(n, c.get("p", 6))
    kind = c["kind"]
    if exact:
        eb = F.exact_bins(X)
        Xb = eb.bin(X)
    else:
        edges, ne = F.bin_edges(X)
        Xb = F.bin_matrix(X, edges, ne, None).numpy()
    ycls = (y > np.median(y)).astype(np.uint8) if kind == 0 else None
    r1 = y if kind == 1 else (w - w.mean() if kind == 2 else None)
    r2 = (y - y.mean()) if kind == 2 else None
    kw = {k: v for k, v in c.items() if k not in ("kind", "p")}
    if exact:
        eng = F.fit_forest(X, kind, y=ycls, r1=r1, r2=r2, ntree=ntree, seed=11,
                           tree_offset=t0, backend=backend, splits="exact", edges=eb, **kw)
    elif backend == "gpu":
        import torch
        Xdev = torch.from_numpy(Xb).cuda()
        eng = F.fit_forest_binned(Xdev, (edges, ne), kind, y=ycls, r1=r1, r2=r2, ntree=ntree,
                                  seed=11, tree_offset=t0, **kw)
    else:
        eng = F.fit_forest_binned(Xb, (edges, ne), kind, y=ycls, r1=r1, r2=r2, ntree=ntree,
                                  seed=11, tree_offset=t0, **kw)
    P = R.Params(kind=kind, seed=11, **kw)
    ref = R.grow_forest(Xb, P, ntree, y=ycls, r1=None if r1 is None else F.to_fix(r1),
                        r2=None if r2 is None else F.to_fix(r2), t0=t0,
                        exact=eb if exact else None)
    return eng, ref, Xb


def assert_same_trees(eng, ref):
    feat, thr, left, val, nn = eng.tree_arrays()
    cap = eng.cap
    n = eng.params.n
    inbag = eng.inbag.cpu().numpy() if hasattr(eng.inbag, "cpu") else np.asarray(eng.inbag)
    est = None if eng.est is None else (eng.est.cpu().numpy() if hasattr(eng.est, "cpu")
                                        else np.asarray(eng.est))
    for t, tr in enumerate(ref):
        m = tr["nnodes"]
        assert int(nn[t]) == m, (t, int(nn[t]), m)
        s = slice(t * cap, t * cap + m)
        np.testing.assert_array_equal(feat[s], tr["feat"])
        inner = tr["feat"] >= 0
        np.testing.assert_array_equal(thr[s][inner], tr["thr"][inner])
        np.testing.assert_array_equal(left[s][inner], tr["left"][inner])
        np.testing.assert_array_equal(val[s], tr["val"])          # bits, not tolerance
        np.testing.assert_array_equal(inbag[t * n:(t + 1) * n], tr["inbag"])
        if "est" in tr:
            np.testing.assert_array_equal(est.reshape(-1, 5)[s], tr["est"])


@pytest.mark.parametrize("name", sorted(CASES))
def test_cpu_engine_equals_numpy_oracle(name):
    eng, ref, _ = _fit_both(name)
    assert max(tr["nnodes"] for tr in ref) > 7                   # real trees, not stumps
    assert_same_trees(eng, ref)


@pytest.mark.parametrize("name", sorted(CASES))
def test_cpu_exact_split_engine_equals_numpy_oracle(name):
    """Exact-split mode (value-rank bins): randomForest midpoint thresholds, grf lower-value
    thresholds with little bags and honesty."""
    eng, ref, _ = _fit_both(name, exact=True)
    assert max(tr["nnodes"] for tr in ref) > 7
    assert_same_trees(eng, ref)


def test_tree_offset_keys_the_streams():
    """A tree-parallel shard (t0 > 0) grows the trees t0.. of the full forest."""
    eng, ref, _ = _fit_both("grf_causal", ntree=2, t0=5)
    assert_same_trees(eng, ref)


def test_oracle_predictions_match_engine():
    """randomForest vote share / mean over OOB trees from the oracle's own tree walk (the
    engines sum each tree's term rounded to 2^-32 fixed point: within ntree * 2^-33)."""
    for name in ("rf_class", "rf_reg"):
        eng, ref, Xb = _fit_both(name, ntree=6)
        got = eng.predict_raw(None, oob=True)
        want = R.predict_mean(ref, Xb, oob=True)
        ok = np.isfinite(want)
        assert ok.sum() > 100
        np.testing.assert_allclose(got[ok], want[ok], rtol=0, atol=6 * 2.0 ** -33)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_per_tree_kernel_equals_numpy_oracle(gpu, name, monkeypatch):
    monkeypatch.setenv("ATE_FOREST_ENGINE", "tree")
    eng, ref, _ = _fit_both(name, backend="gpu")
    assert eng.backend == "gpu"
    assert_same_trees(eng, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["rf_class", "rf_reg"])
def test_gpu_level_engine_equals_numpy_oracle(gpu, name, monkeypatch):
    """The GPU-wide level engine (csrc/forest_level.hip, randomForest sampling)."""
    monkeypatch.setenv("ATE_FOREST_ENGINE", "level")
    eng, ref, _ = _fit_both(name, backend="gpu")
    assert_same_trees(eng, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_exact_split_kernel_equals_numpy_oracle(gpu, name):
    """csrc/forest_exact.hip against the oracle."""
    eng, ref, _ = _fit_both(name, backend="gpu", exact=True)
    assert eng.backend == "gpu"
    assert_same_trees(eng, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["rf_class", "rf_reg", "grf_causal", "grf_causal_m12",
                                  "rf_reg_m10"])
def test_gpu_exact_split_kernel_large_nodes_equals_oracle(gpu, name):
    """n = 3000: workgroup-level nodes (> 256 rows), wave-level list nodes and lane-per-row
    nodes (<= 64 rows, whose lists are never partitioned) in the same trees."""
    eng, ref, _ = _fit_both(name, backend="gpu", exact=True, ntree=2, n=3000)
    assert max(tr["nnodes"] for tr in ref) > 200
    assert_same_trees(eng, ref)


def test_cpu_exact_split_engine_large_nodes_equals_oracle():
    eng, ref, _ = _fit_both("rf_reg", exact=True, ntree=1, n=3000)
    assert_same_trees(eng, ref)


@pytest.mark.parametrize("n,group,sf,honesty", [(160, 2, 0.5, True), (161, 2, 0.5, False),
                                                (500, 1, 0.5, True), (333, 1, 0.6, True),
                                                (777, 2, 0.3, True), (50, 4, 0.5, True)])
def test_exact_mcap_is_the_in_bag_count(n, group, sf, honesty):
    """models/forest.exact_mcap (the per-position scratch size of csrc/forest_exact.hip) equals
    the J1 row count the oracle's grf sampling draws for every tree."""
    P = R.Params(kind=2, sampling=1, group=group, sample_fraction=sf, honesty=honesty, seed=7)
    for tg in range(5):
        w, _, _ = R._tree_rows(P, n, tg)
        assert int((w > 0).sum()) == F.exact_mcap(n, 1, group, sf, honesty)
    assert F.exact_mcap(n, 0, 1, 0.5, False) == n
