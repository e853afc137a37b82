"""Property tests (SURVEY.md §4.2 "Property (hypothesis)"): invariances of the float64
oracle and the device orchestration, checked over hypothesis-generated small inputs.

* naive ATE: row-permutation and outcome-shift invariance (E1);
* OLS: outcome-scale equivariance of the W coefficient and its SE, invariance to
  rescaling a covariate, R's aliasing of a duplicated column (E2, N1 rank rule);
* AIPW with zero outcome models is the Horvitz-Thompson IPW mean (E8/E9 algebra);
* glmnet covariance-mode CD: KKT conditions at every lambda of the path (N3; for the
  gaussian family glmnet standardises y, so the ridge part acts on b / sd(y));
* binning: a binary feature's histogram split is the exact split (K11-K13);
* GBDT: fixed-point histograms make the trees independent of the row order (K12);
* Philox: counter RNG draws and fold ids do not depend on how rows are chunked or
  sharded (K10, world-size invariance).
"""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from ate_replication_causalml_amd.models import forest as F
from ate_replication_causalml_amd.models import gbdt as G
from ate_replication_causalml_amd.parallel import rng
from ate_replication_causalml_amd.reference import estimators as E
from ate_replication_causalml_amd.reference import glmnet as GN
from ate_replication_causalml_amd.reference.linear import lm_fit

SETTINGS = settings(max_examples=25, deadline=None,
                    suppress_health_check=[HealthCheck.too_slow])
seeds = st.integers(min_value=0, max_value=2 ** 31 - 1)


def _panel(seed, n=200, p=4):
    r = np.random.default_rng(seed)
    X = r.normal(size=(n, p))
    W = (r.random(n) < 0.5).astype(float)
    W[:2] = [0.0, 1.0]
    Y = X @ r.normal(size=p) + 0.7 * W + r.normal(size=n)
    return X, W, Y


@SETTINGS
@given(seed=seeds, shift=st.floats(-100, 100))
def test_naive_permutation_and_shift_invariant(seed, shift):
    _, W, Y = _panel(seed)
    a = E.naive(Y, W)
    perm = np.random.default_rng(seed + 1).permutation(len(Y))
    b = E.naive(Y[perm] + shift, W[perm])
    assert b.ate == pytest.approx(a.ate, abs=1e-9)
    assert b.se == pytest.approx(a.se, rel=1e-9)
    assert a.ate == pytest.approx(Y[W == 1].mean() - Y[W == 0].mean(), abs=1e-12)


@SETTINGS
@given(seed=seeds, c=st.floats(0.01, 100), d=st.floats(0.01, 100))
def test_ols_scale_equivariance(seed, c, d):
    X, W, Y = _panel(seed)
    a = E.ols(Y, W, X)
    b = E.ols(c * Y, W, X)
    assert b.ate == pytest.approx(c * a.ate, rel=1e-8, abs=1e-10)
    assert b.se == pytest.approx(c * a.se, rel=1e-8)
    X2 = X.copy()
    X2[:, 0] *= d                                   # rescaled covariate: same W effect
    e = E.ols(Y, W, X2)
    assert e.ate == pytest.approx(a.ate, rel=1e-8, abs=1e-10)
    assert e.se == pytest.approx(a.se, rel=1e-8)


@SETTINGS
@given(seed=seeds)
def test_ols_duplicate_column_is_aliased(seed):
    X, W, Y = _panel(seed)
    Xd = np.column_stack([X, X[:, 1]])
    fit = lm_fit(np.column_stack([Xd, W]), Y)
    assert fit.aliased[1 + Xd.shape[1] - 1]         # the later copy (after intercept)
    assert np.isnan(fit.coef[Xd.shape[1]])
    ref = lm_fit(np.column_stack([X, W]), Y)
    assert fit.coef[-1] == pytest.approx(ref.coef[-1], rel=1e-9)
    assert fit.se[-1] == pytest.approx(ref.se[-1], rel=1e-9)


@SETTINGS
@given(seed=seeds)
def test_aipw_with_zero_outcome_models_is_ipw(seed):
    X, W, Y = _panel(seed)
    p = np.clip(1 / (1 + np.exp(-X[:, 0])), 0.05, 0.95)
    z = np.zeros_like(Y)
    tau = E.aipw_point(W, Y, p, z, z, compat="textbook")
    ht = np.mean(W * Y / p - (1 - W) * Y / (1 - p))
    assert tau == pytest.approx(ht, rel=1e-12, abs=1e-12)


@SETTINGS
@given(seed=seeds, alpha=st.sampled_from([1.0, 0.9, 0.5]))
def test_glmnet_path_satisfies_kkt(seed, alpha):
    r = np.random.default_rng(seed)
    n, p = 120, 6
    X = r.normal(size=(n, p)) * r.uniform(0.5, 3.0, size=p)
    y = X[:, 0] - 0.5 * X[:, 2] + r.normal(size=n)
    path = GN.glmnet(X, y, alpha=alpha, nlambda=30)
    xm, xs = X.mean(0), X.std(0)                       # glmnet: 1/n variance
    ys = y.std()              # gaussian glmnet scales y by ys, so the ridge term is b/ys
    for lam, a0, beta in zip(path.lambdas, path.a0, path.beta):
        res = y - a0 - X @ beta
        grad = ((X - xm) / xs).T @ res / n             # standardized coordinates
        b = beta * xs
        # coordinate descent stops on an objective-change threshold (1e-7 x null
        # deviance), so the gradient residual carries an absolute floor near the tail
        tol = 2e-3 * lam + 5e-5
        for j in range(p):
            if b[j] != 0:
                want = lam * (alpha * np.sign(b[j]) + (1 - alpha) * b[j] / ys)
                assert grad[j] == pytest.approx(want, abs=tol * 5 + 1e-3 * abs(want))
            else:
                assert abs(grad[j]) <= lam * alpha + tol


@SETTINGS
@given(seed=seeds)
def test_binary_feature_histogram_split_is_exact(seed):
    r = np.random.default_rng(seed)
    x = (r.random(300) < r.uniform(0.2, 0.8)).astype(float)
    X = np.column_stack([x, r.normal(size=300)])
    edges, ne = F.bin_edges(X)
    assert ne[0] == 1 and edges[0, 0] == 0.5
    b = F.bin_matrix(X, edges, ne).numpy()
    np.testing.assert_array_equal(b[0], x.astype(np.uint8))   # bin <= 0  <=>  x <= 0.5


@settings(max_examples=8, deadline=None)
@given(seed=seeds)
def test_gbdt_trees_independent_of_row_order(seed):
    r = np.random.default_rng(seed)
    X = r.normal(size=(400, 3))
    y = np.sin(X[:, 0]) + 0.3 * X[:, 1] + 0.1 * r.normal(size=400)
    edges = F.bin_edges(X)
    a = G.fit_gbdt(X, y, n_trees=3, depth=3, backend="cpu", edges=edges)
    perm = r.permutation(400)
    b = G.fit_gbdt(X[perm], y[perm], n_trees=3, depth=3, backend="cpu", edges=edges)
    np.testing.assert_array_equal(a.feat, b.feat)
    np.testing.assert_array_equal(a.thr[a.feat >= 0], b.thr[b.feat >= 0])
    np.testing.assert_array_equal(a.value, b.value)


@SETTINGS
@given(seed=seeds, n=st.integers(10, 500), cut=st.integers(1, 9))
def test_philox_draws_and_folds_are_chunking_invariant(seed, n, cut):
    idx = np.arange(n, dtype=np.uint64)
    full = rng.random_u32(seed, rng.P_FOLD, 3, idx)
    k = n * cut // 10
    parts = np.concatenate([rng.random_u32(seed, rng.P_FOLD, 3, idx[:k]),
                            rng.random_u32(seed, rng.P_FOLD, 3, idx[k:])])
    np.testing.assert_array_equal(full, parts)
    f = rng.fold_ids(n, 5, seed, 2)
    assert np.bincount(f, minlength=5).max() - np.bincount(f, minlength=5).min() <= 1
