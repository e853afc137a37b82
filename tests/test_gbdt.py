"""Histogram GBDT (models/gbdt.py, reference/gbdt.py): fit quality, determinism,
row-sharded training (C04 all-reduce) equal to single-device, DML with GBDT nuisances."""
import numpy as np
import pytest

from ate_replication_causalml_amd.models import gbdt as G
from ate_replication_causalml_amd.parallel.comm import run_simulated
from ate_replication_causalml_amd.parallel.dist import DistContext


def _data(n=3000, seed=0):
    r = np.random.default_rng(seed)
    X = r.normal(size=(n, 5))
    y = np.sin(X[:, 0]) + 0.5 * (X[:, 1] > 0) + 0.1 * r.normal(size=n)
    return X, y


def test_gbdt_fits_and_generalises():
    X, y = _data()
    tr = np.arange(len(y)) % 5 != 0
    m = G.fit_gbdt(X, y, n_trees=40, depth=4, lr=0.2, train=tr, backend="cpu")
    f = m.predict(X)
    assert np.mean((f - y)[~tr] ** 2) < 0.05 * y.var() + 0.02
    yb = (y > 0.3).astype(float)
    mb = G.fit_gbdt(X, yb, loss="logistic", n_trees=30, depth=3, lr=0.3, backend="cpu")
    assert np.mean((mb.predict(X, response=True) > 0.5) == yb) > 0.9


def test_gbdt_leaf_values_are_newton_steps():
    """One depth-1 tree with lr=1, lam=0: leaves hold -mean residual of their side."""
    X, y = _data(500, 3)
    m = G.fit_gbdt(X, y, n_trees=1, depth=1, lr=1.0, lam=0.0, backend="cpu")
    f = m.predict(X)
    left = f < np.median(f) if len(np.unique(f)) == 2 else None
    assert len(np.unique(np.round(f, 12))) == 2
    for v in np.unique(np.round(f, 12)):
        sel = np.isclose(f, v)
        assert np.mean(y[sel]) == pytest.approx(v, abs=1e-7)


@pytest.mark.parametrize("world", [2, 3, 4])
def test_gbdt_row_sharded_equals_single(world):
    """Row shards (C04 int64 histogram all-reduce, exact base, GLOBAL edge sample) grow
    the single-device trees bit for bit -- the edges here come from global_bin_edges on
    each rank's shard, not a pinned host array."""
    X, y = _data(1200, 1)
    m1 = G.fit_gbdt(X, y, n_trees=8, depth=3, backend="cpu")

    def fn(comm):
        d = DistContext.for_rank(comm, len(y))
        return G.fit_gbdt(d.local(X), d.local(y), n_trees=8, depth=3, backend="cpu", dist=d)

    for m in run_simulated(world, fn):
        np.testing.assert_array_equal(m.edges[0], m1.edges[0])
        np.testing.assert_array_equal(m.feat, m1.feat)
        np.testing.assert_array_equal(m.thr, m1.thr)
        np.testing.assert_array_equal(m.value, m1.value)
        assert m.base == m1.base


def test_c04_slice_geometry():
    class D:
        def __init__(self, w):
            self.world, self.rank = w, 0
    assert G.c04_slices(5, None) == (1, 5)
    assert G.c04_slices(5, D(1)) == (1, 5)
    assert G.c04_slices(5, D(2)) == (2, 3)
    assert G.c04_slices(5, D(3)) == (3, 2)
    assert G.c04_slices(5, D(4)) == (1, 5)          # rank 3's slice would be empty
    assert G.c04_slices(2000, D(8)) == (8, 250)


@pytest.mark.parametrize("world,mode", [(2, "sliced"), (3, "sliced"), (3, "allreduce")])
def test_gbdt_feature_sliced_c04_equals_single(world, mode, monkeypatch):
    """Feature-sliced C04 (reduce-scatter of each level's histograms, split search on the
    rank's slice, all-gather of the per-node candidates): the signal sits in features owned
    by different ranks (first and last), so the winning split comes from any rank; the
    trees equal the single-device ones bit for bit, and so do those of the all-reduce
    scheme (ATE_GBDT_C04=allreduce)."""
    if mode == "allreduce":
        monkeypatch.setenv("ATE_GBDT_C04", "allreduce")
    r = np.random.default_rng(7)
    X = r.normal(size=(1500, 7))
    y = np.sin(X[:, 6]) + 0.7 * (X[:, 0] > 0.3) - 0.4 * X[:, 3] + 0.1 * r.normal(size=1500)
    m1 = G.fit_gbdt(X, y, n_trees=6, depth=4, backend="cpu")
    calls = []
    orig = G.SlicedC04.scatter

    def spy(self, hist):
        calls.append(self.pl)
        return orig(self, hist)
    monkeypatch.setattr(G.SlicedC04, "scatter", spy)

    def fn(comm):
        d = DistContext.for_rank(comm, len(y))
        return G.fit_gbdt(d.local(X), d.local(y), n_trees=6, depth=4, backend="cpu", dist=d)

    for m in run_simulated(world, fn):
        np.testing.assert_array_equal(m.feat, m1.feat)
        np.testing.assert_array_equal(m.thr, m1.thr)
        np.testing.assert_array_equal(m.value, m1.value)
    assert set(m1.feat[m1.feat >= 0].tolist()) >= {0, 6}
    if mode == "sliced":
        pw = -(-7 // world)
        assert sorted(set(calls)) == sorted({pw, 7 - (world - 1) * pw})
    else:
        assert not calls


def test_global_edges_equal_single_device_edges_large_n():
    """n > the edge sample: each rank's rows of the global strided sample, gathered, give
    exactly sample_bin_edges of the whole matrix."""
    X, _ = _data(5000, 2)
    want = G.sample_bin_edges(X, rows=701)

    def fn(comm):
        d = DistContext.for_rank(comm, len(X))
        return G.global_bin_edges(d.local(X), d, rows=701)

    for e, ne in run_simulated(3, fn):
        np.testing.assert_array_equal(e, want[0])
        np.testing.assert_array_equal(ne, want[1])


@pytest.mark.parametrize("world", [2, 4])
def test_dml_gbdt_sharded_bitwise_equals_single(tutorial, world):
    """DML-GBDT on row shards: exact histograms + exact score moments -> the ATE and SE
    are the SAME BITS as one process (rtol=0)."""
    from ate_replication_causalml_amd.estimators.boosting import dml_plr_gbdt
    _, m, _ = tutorial
    kw = dict(n_trees=5, depth=3, device="cpu")
    a = dml_plr_gbdt(m.Y, m.W, m.X, **kw)

    def fn(comm):
        d = DistContext.for_rank(comm, len(m.Y))
        return dml_plr_gbdt(d.local(m.Y), d.local(m.W), d.local(m.X), dist=d, **kw)
    for b in run_simulated(world, fn):
        assert b.ate == a.ate and b.se == a.se


def test_dml_gbdt_checkpoint_resume(tutorial, tmp_path, monkeypatch):
    """Kill the cross-fit after fold 2, resume from the checkpoint: the finished folds are
    loaded (not refit) and the ATE / SE are bitwise identical to an uninterrupted run."""
    from ate_replication_causalml_amd.estimators import boosting as EB
    from ate_replication_causalml_amd.utils.checkpoint import Checkpoint
    _, m, _ = tutorial
    kw = dict(n_trees=4, depth=3, device="cpu")
    want = EB.dml_plr_gbdt(m.Y, m.W, m.X, **kw)
    real = G.fit_gbdt
    calls = {"n": 0}

    class Killed(RuntimeError):
        pass

    def dying(*a, **k):
        calls["n"] += 1
        if calls["n"] > 6:                      # folds 0-2 done (2 fits each), die in fold 3
            raise Killed()
        return real(*a, **k)
    monkeypatch.setattr(G, "fit_gbdt", dying)
    ck = Checkpoint(tmp_path, {"cfg": "dml_gbdt"})
    with pytest.raises(Killed):
        EB.dml_plr_gbdt(m.Y, m.W, m.X, checkpoint=ck, **kw)
    assert sorted(p.name.split(".")[0] for p in tmp_path.glob("*.npz")) == \
        ["dml_gbdt_fold0", "dml_gbdt_fold1", "dml_gbdt_fold2"]
    calls["n"] = -10**9                          # no more deaths; count the refits
    got = EB.dml_plr_gbdt(m.Y, m.W, m.X, checkpoint=ck, **kw)
    assert calls["n"] == -10**9 + 4              # only folds 3 and 4 were fitted
    assert got.ate == want.ate and got.se == want.se
