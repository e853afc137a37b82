"""Independent checks of the causal-forest spec (grf::causal_forest, ate_replication.Rmd:250-270)
against known truth instead of the implementation's own twin:

* honesty: every tree's estimation statistics come from the J2 half of its subsample only
  (counts per node, children summing to their parent);
* the little-bag variance debiaser equals the normal posterior mean computed with scipy;
* CATE recovery and pointwise interval coverage on the heterogeneous surface of Wager &
  Athey (2018, Sec. 5.1), tau(x) = zeta(x1) zeta(x2), zeta(u) = 1 + 1 / (1 + e^{-20 (u - 1/3)});
* variance calibration under a null effect over independent replicate data sets.
All on the host engine (the GPU engine equals it bit for bit: tests/test_forest_gpu.py).
"""
import ctypes

import numpy as np
import pytest

from ate_replication_causalml_amd import _native
from ate_replication_causalml_amd.models import forest as F


def _zeta(u):
    return 1 + 1 / (1 + np.exp(-20 * (u - 1 / 3)))


def test_grf_debias_is_the_normal_posterior_mean():
    """forest_common.hpp grf_debias (built from +,-,*,/ so host and device agree bitwise) ==
    est + se * phi(r) / Phi(r) with scipy's density and CDF."""
    from scipy.stats import norm
    f = _native.cpu().atecpu_grf_debias
    f.restype = ctypes.c_double
    f.argtypes = [ctypes.c_double] * 3
    r = np.random.default_rng(0)
    cases = [(1.0, 0.5, 100), (0.5, 1.0, 100), (1e-3, 1e-2, 1000), (1.0, 1.0, 50),
             (2.0, 0.1, 10), (0.01, 10.0, 1000), (3e-5, 1e-5, 500)]
    cases += [(float(a), float(b), float(g)) for a, b, g in
              zip(r.exponential(size=40), r.exponential(size=40), r.integers(2, 2000, 40))]
    for b, nz, g in cases:
        est = b - nz
        se = max(b, nz) * np.sqrt(2 / g)
        q = est / se
        want = est + se * np.exp(norm.logpdf(q) - norm.logcdf(q))
        got = f(b, nz, g)
        assert got > 0
        # the formula itself cancels (est + se * m with m ~ -q) in the far tail
        assert abs(got - want) <= 1e-13 * (abs(est) + se) + 1e-12 * abs(want), (b, nz, g)
    assert f(0.0, 0.0, 10) == 0.0


@pytest.mark.parametrize("honesty", [True, False])
def test_estimation_statistics_come_from_the_honest_half(honesty):
    r = np.random.default_rng(3)
    n = 1200
    X = r.normal(size=(n, 5))
    W = (r.uniform(size=n) < 0.5).astype(float)
    Y = X[:, 0] + W * (X[:, 1] > 0) + r.normal(size=n)
    T = 20
    cf = F.causal_forest(X, Y, W, num_trees=T, seed=5, backend="cpu", honesty=honesty)
    fo = cf.forest
    cap = fo.cap
    est = np.asarray(fo.est).reshape(T, cap, 5)
    inbag = np.asarray(fo.inbag).reshape(T, n).astype(bool)
    feat = np.asarray(fo.feat).reshape(T, cap)
    left = np.asarray(fo.left).reshape(T, cap)
    nn = np.asarray(fo.nnodes).reshape(T)
    for t in range(T):
        s = int(inbag[t].sum())
        # little bags of 2: the group's half-sample H (n/2 rows) is every tree's subsample
        assert s == n // 2
        # J2 = the subsample minus its random half J1 (honesty), else the whole subsample
        assert est[t, 0, 0] == (s - s // 2 if honesty else s)
        for v in range(nn[t]):
            if feat[t, v] >= 0:
                c = left[t, v]
                assert est[t, v, 0] == est[t, c, 0] + est[t, c + 1, 0]
                # sums of W~ (fixed point) split the same way
                assert est[t, v, 1] == est[t, c, 1] + est[t, c + 1, 1]


def test_cate_surface_and_interval_coverage():
    """Wager & Athey (2018) Sec. 5.1 surface, d = 4, n = 3000, randomised W: the forest
    tracks tau(x) on new points and its little-bag intervals cover near nominally
    (grf's Bayes-debiased variance; a clamp at zero gave 0.69 here)."""
    r = np.random.default_rng(0)
    n, d = 3000, 4
    X = r.uniform(size=(n, d))
    W = (r.uniform(size=n) < 0.5).astype(float)
    Y = _zeta(X[:, 0]) * _zeta(X[:, 1]) * W + r.normal(size=n)
    Xt = r.uniform(size=(300, d))
    taut = _zeta(Xt[:, 0]) * _zeta(Xt[:, 1])
    cf = F.causal_forest(X, Y, W, num_trees=1000, seed=3, backend="cpu")
    out = cf.forest.predict_raw(Xt)
    th, v = out[:, 0], out[:, 1]
    assert np.corrcoef(th, taut)[0, 1] > 0.93
    assert np.sqrt(np.mean((th - taut) ** 2)) < 0.35 * taut.std() + 0.05
    assert np.all(v > 0)
    cover = np.mean(np.abs(th - taut) <= 1.96 * np.sqrt(v))
    assert 0.8 <= cover <= 1.0, cover


def test_variance_is_calibrated_under_a_null_effect():
    """tau = 0: over independent data sets the forest's variance estimate at fixed test
    points matches the replicate variance of its estimate (grf's little bags are slightly
    conservative at this size), and the 95% intervals cover zero."""
    n, d, R = 2000, 4, 16
    Xt = np.random.default_rng(99).uniform(size=(100, d))
    ths, vs = [], []
    for rep in range(R):
        r = np.random.default_rng(rep)
        X = r.uniform(size=(n, d))
        W = (r.uniform(size=n) < 0.5).astype(float)
        Y = X[:, 0] + r.normal(size=n)
        cf = F.causal_forest(X, Y, W, num_trees=600, seed=rep + 1, backend="cpu")
        out = cf.forest.predict_raw(Xt)
        ths.append(out[:, 0])
        vs.append(out[:, 1])
    ths, vs = np.array(ths), np.array(vs)
    ratio = vs.mean() / ths.var(0, ddof=1).mean()
    assert 0.6 < ratio < 3.0, ratio
    assert abs(ths.mean()) < 3 * np.sqrt(vs.mean() / (R * 10))
    cover = np.mean(np.abs(ths) <= 1.96 * np.sqrt(vs))
    assert cover >= 0.88, cover


def _stabilize_data():
    """One feature x = 0..399 (distinct values); below x = 30 a strong effect but only 2 of
    the 30 rows on the treated side of the node's mean W~, so the unconstrained best root
    split (x <= 29) leaves the left child 2 treated-side rows."""
    n = 400
    x = np.arange(n, dtype=float)
    r = np.random.default_rng(1)
    wt = np.where(np.arange(n) % 2 == 0, 0.5, -0.5)
    wt[:30] = -0.5
    wt[[3, 17]] = 0.5
    yt = np.where(x < 30, 3.0 * wt, 0.0) + 0.01 * r.normal(size=n)
    return x[:, None], wt - wt.mean(), yt - yt.mean()


def _root_best(x, wt, yt, minc, rule):
    """Brute-force root split on the pseudo-outcomes: 'arm1' = >= 1 row on each side of the
    mean W~ per child (the previous rule), 'stabilize' = >= minc (grf stabilize.splits)."""
    wbar, ybar = wt.mean(), yt.mean()
    cww = (wt * wt).mean() - wbar * wbar
    tau = ((wt * yt).mean() - wbar * ybar) / cww
    rho = (wt - wbar) * ((yt - ybar) - tau * (wt - wbar)) / cww
    o = np.argsort(x[:, 0], kind="stable")
    big = (wt >= wbar)[o]
    n = len(o)
    best, arg = -np.inf, None
    for k in range(1, n):
        nl, nr = k, n - k
        lt, rt = int(big[:k].sum()), int(big[k:].sum())
        need = 1 if rule == "arm1" else minc
        if nl < minc or nr < minc or lt < need or nl - lt < need or rt < need or nr - rt < need:
            continue
        sl, sr = rho[o][:k].sum(), rho[o][k:].sum()
        c = sl * sl / nl + sr * sr / nr
        if c > best:
            best, arg = c, k - 1          # threshold rank: x <= arg goes left
    return arg


@pytest.mark.parametrize("splits", ["exact", "binned"])
def test_stabilize_splits_rule_pins_the_root(splits):
    """grf's stabilize.splits = TRUE (forest_common.hpp kind 2): with alpha = 0.05 at a
    400-row root each child needs >= 20 rows on both sides of the mean W~. The old ">= 1
    row per side" rule would split at x <= 29 (two treated-side rows on the left); the
    engine splits where the new rule's best is, and the oracle grows the same tree."""
    from ate_replication_causalml_amd.reference import forest as R
    X, wt, yt = _stabilize_data()
    old = _root_best(X, wt, yt, 20, "arm1")
    new = _root_best(X, wt, yt, 20, "stabilize")
    assert old == 29 and new != old
    kw = dict(ntree=1, mtry=1, min_node=5, sampling=1, honesty=False, group=1,
              mtry_poisson=False, alpha=0.05, sample_fraction=1.0, seed=3)
    eng = F.fit_forest(X, F.KIND_CAUSAL, r1=wt, r2=yt, backend="cpu", splits=splits, **kw)
    feat, thr, left, val, nn = eng.tree_arrays()
    assert feat[0] == 0
    if splits == "exact":
        assert thr[0] == new                       # value rank = x for distinct integers
    else:
        edges, ne = eng.edges, eng.nedges
        # the binned engine's root threshold bin covers x <= new (400 distinct values in
        # 256 quantile bins: the admissible boundary nearest the exact one)
        cut = edges[0, thr[0]]
        assert abs(cut - (new + 0.5)) <= 2.0
        assert cut > 29.5 + 1
    # the oracle (reference/forest.py) grows the same tree from the written spec
    if splits == "exact":
        eb = F.exact_bins(X)
        Xb = eb.bin(X)
    else:
        Xb = F.bin_matrix(X, eng.edges, eng.nedges, None).numpy()
    P = R.Params(kind=2, sampling=1, mtry=1, min_node=5, honesty=False, group=1,
                 mtry_poisson=False, alpha=0.05, sample_fraction=1.0, seed=3)
    ref = R.grow_forest(Xb, P, 1, r1=F.to_fix(wt), r2=F.to_fix(yt),
                        exact=eb if splits == "exact" else None)
    assert int(nn[0]) == ref[0]["nnodes"]
    np.testing.assert_array_equal(thr[:ref[0]["nnodes"]][ref[0]["feat"] >= 0],
                                  ref[0]["thr"][ref[0]["feat"] >= 0])
