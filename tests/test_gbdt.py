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


@pytest.mark.parametrize("world", [2, 3])
def test_gbdt_row_sharded_equals_single(world):
    X, y = _data(1200, 1)
    edges = G.global_bin_edges(X, None)
    m1 = G.fit_gbdt(X, y, n_trees=8, depth=3, backend="cpu", edges=edges)

    def fn(comm):
        d = DistContext.for_rank(comm, len(y))
        m = G.fit_gbdt(d.local(X), d.local(y), n_trees=8, depth=3, backend="cpu", edges=edges,
                       dist=d)
        return m

    for m in run_simulated(world, fn):
        np.testing.assert_array_equal(m.feat, m1.feat)
        np.testing.assert_array_equal(m.thr, m1.thr)
        np.testing.assert_allclose(m.value, m1.value, rtol=0, atol=0)


def test_dml_gbdt_sharded_equals_single(tutorial):
    from ate_replication_causalml_amd.estimators.boosting import dml_plr_gbdt
    _, m, _ = tutorial
    kw = dict(n_trees=5, depth=3, device="cpu")
    a = dml_plr_gbdt(m.Y, m.W, m.X, **kw)
    # global edges differ from single-device edges only through the sample; pin them equal
    def fn(comm):
        d = DistContext.for_rank(comm, len(m.Y))
        return dml_plr_gbdt(d.local(m.Y), d.local(m.W), d.local(m.X), dist=d, **kw)
    for b in run_simulated(2, fn):
        assert b.ate == pytest.approx(a.ate, rel=1e-9)
        assert b.se == pytest.approx(a.se, rel=1e-9)
