"""CPU tests of the float64 reference path (T-ref) against closed forms and
scikit-learn, plus the reference-quirk mechanics."""
import numpy as np
import pytest

from ate_replication_causalml_amd.data import dgp, selection
from ate_replication_causalml_amd.parallel import rng
from ate_replication_causalml_amd.reference import estimators as E
from ate_replication_causalml_amd.reference import glmnet as G
from ate_replication_causalml_amd.reference.linear import glm_logit, lm_fit


def test_philox_known_answer():
    # Random123 known-answer test for philox4x32-10: counter=0, key=0
    out = rng.philox4x32(0, 0, 0, 0, 0, 0)
    assert [int(v) for v in out] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    out = rng.philox4x32(0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF)
    assert [int(v) for v in out] == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]


def test_fold_ids_balanced_and_deterministic():
    f1 = rng.fold_ids(1003, 10, seed=5)
    f2 = rng.fold_ids(1003, 10, seed=5)
    assert (f1 == f2).all()
    c = np.bincount(f1)
    assert c.max() - c.min() <= 1
    assert not (rng.fold_ids(1003, 10, seed=6) == f1).all()


def test_bootstrap_counts_sum():
    c = rng.bootstrap_counts(500, 1, rng.P_BOOT, 3)
    assert c.sum() == 500 and (c >= 0).all()


def test_selection_transform_rules():
    names = dgp.COVARIATES
    X = np.zeros((8, len(names)))
    col = {n: i for i, n in enumerate(names)}
    X[:, col["p2004"]] = 1
    # row 0 treated with only p2004==1: reference rule omits p2004 -> not dropped (Q17)
    W = np.array([1, 1, 1, 1, 0, 0, 0, 0], float)
    X[1, col["g2000"]] = 1
    X[2, col["city"]] = 3
    X[3, col["yob"]] = 2.5
    for r in range(4, 8):
        X[r, [col[c] for c in ["g2000", "g2002", "p2000", "p2002", "p2004"]]] = 1
    X[4, col["g2002"]] = 0
    X[5, col["city"]] = -3
    dt, dc = selection.selection_masks(X, names, "reference")
    assert list(dt[:4]) == [False, True, True, True]
    dt2, _ = selection.selection_masks(X, names, "textbook")
    assert dt2[0]
    assert list(dc[4:]) == [True, True, False, False]
    # first round(0.85*k) in row order (Q18): k=3 treated -> round(2.55)=3
    drop = selection.drop_indices(X, W, names)
    assert list(drop) == [1, 2, 3, 4, 5]


def test_tutorial_shape():
    d = dgp.make_tutorial_data(n=4000, seed=3)
    assert d.X.shape == (4000, 21)
    assert set(np.unique(d.W)) == {0.0, 1.0} and set(np.unique(d.Y)) == {0.0, 1.0}
    cts = d.X[:, :15]
    assert np.allclose(cts.mean(0), 0, atol=1e-12) and np.allclose(cts.std(0, ddof=1), 1)


def test_lm_matches_lstsq_and_se():
    rs = np.random.RandomState(0)
    X = rs.randn(300, 4)
    y = X @ [1, 2, 0, -1] + rs.randn(300)
    f = lm_fit(X, y)
    A = np.column_stack([np.ones(300), X])
    b = np.linalg.lstsq(A, y, rcond=None)[0]
    assert np.allclose(f.coef, b)
    s2 = np.sum((y - A @ b) ** 2) / (300 - 5)
    assert np.allclose(f.se, np.sqrt(s2 * np.diag(np.linalg.inv(A.T @ A))))


def test_lm_aliasing_column_order():
    rs = np.random.RandomState(1)
    X = rs.randn(200, 5)
    X[:, 3] = X[:, 0] - X[:, 1]      # aliased (later column gets NA)
    X[:, 4] = 2 * X[:, 2]
    f = lm_fit(X, rs.randn(200))
    assert list(f.aliased) == [False, False, False, False, True, True]
    assert f.rank == 4 and np.isnan(f.coef[4]) and np.isnan(f.se[5])


def test_weighted_lm():
    rs = np.random.RandomState(2)
    x = rs.randn(100)
    y = 1 + 2 * x + rs.randn(100)
    w = rs.rand(100) + 0.5
    f = lm_fit(x, y, weights=w)
    A = np.column_stack([np.ones(100), x])
    b = np.linalg.solve(A.T @ (A * w[:, None]), A.T @ (w * y))
    assert np.allclose(f.coef, b)


def test_glm_logit_vs_sklearn():
    from sklearn.linear_model import LogisticRegression
    rs = np.random.RandomState(3)
    X = rs.randn(1000, 3)
    y = (rs.rand(1000) < 1 / (1 + np.exp(-(X @ [1, -0.5, 0.2] + 0.3)))).astype(float)
    f = glm_logit(X, y)
    m = LogisticRegression(penalty=None, tol=1e-12, max_iter=10000).fit(X, y)
    assert f.converged
    assert np.allclose(f.coef, np.r_[m.intercept_, m.coef_[0]], atol=1e-5)


def test_glmnet_gaussian_vs_sklearn():
    from sklearn.linear_model import Lasso
    rs = np.random.RandomState(0)
    X = rs.randn(800, 12)
    y = X[:, :3] @ [1, -2, 0.5] + rs.randn(800)
    f = G.elnet_gaussian(X, y)
    assert 5 <= len(f.lambdas) <= 100
    assert np.all(np.diff(f.lambdas) < 0)
    assert np.allclose(f.beta[0], 0)      # lambda_max gives the null model
    xm, xs, ym, ys = X.mean(0), X.std(0), y.mean(), y.std()
    for i in (5, 20):
        m = Lasso(alpha=f.lambdas[i] / ys, tol=1e-12, max_iter=100000).fit((X - xm) / xs,
                                                                           (y - ym) / ys)
        assert np.allclose(m.coef_ * ys / xs, f.beta[i], atol=1e-6)


def test_glmnet_unpenalized_factor():
    rs = np.random.RandomState(4)
    X = rs.randn(500, 6)
    y = X[:, 5] * 0.01 + X[:, 0] + rs.randn(500)
    pf = np.r_[np.ones(5), 0.0]
    f = G.elnet_gaussian(X, y, penalty_factor=pf)
    assert f.beta[0, 5] != 0       # unpenalised variable in the model at lambda_max
    assert np.allclose(f.beta[0, :5], 0)


def test_cv_select_rules():
    lam = np.array([1.0, 0.5, 0.25, 0.125])
    raw = np.array([[4.0, 2.0, 1.0, 1.0], [4.0, 2.2, 1.2, 1.4]])
    cvm, cvsd, imin, i1 = G.cv_select(lam, raw, [10, 10])
    assert imin == 2                      # first (largest lambda) attaining the min
    assert i1 == 2 or cvm[i1] <= cvm[imin] + cvsd[imin]


def test_lambda_interp_matches_glmnet_rule():
    lam = np.array([1.0, 0.5, 0.25])
    assert E.lambda_interp(lam, 0.5) == (1, 1, 1.0)
    l, r, f = E.lambda_interp(lam, 0.75)
    assert (l, r) == (0, 1) and abs(f - 0.5) < 1e-12
    assert E.lambda_interp(lam, 5.0)[:2] == (0, 0)


def test_naive_se_uses_n_minus_1(tutorial):
    _, m, _ = tutorial
    r = E.naive(m.Y, m.W)
    y1, y0 = m.Y[m.W == 1], m.Y[m.W == 0]
    se = np.sqrt(y1.var(ddof=1) / (len(y1) - 1) + y0.var(ddof=1) / (len(y0) - 1))
    assert abs(r.se - se) < 1e-15 and abs(r.upper_ci - r.ate - 1.96 * se) < 1e-15


def test_ipw_quirk_design_has_full_frame(tutorial):
    _, m, _ = tutorial
    p = E.propensity_logistic(m.W, m.X)
    d, tau = E.ipw_design(m.Y, m.W, m.X, p, "reference")
    assert d.shape[1] == 21 + 5
    d2, _ = E.ipw_design(m.Y, m.W, m.X, p, "textbook")
    assert d2.shape[1] == 21
    # W*ps - p*ps == ps^2 exactly: lm aliases the last column
    from ate_replication_causalml_amd.reference.linear import lm_fit
    assert lm_fit(d, tau).aliased[-1]


def test_aipw_sign_quirk():
    w = np.array([1.0, 0.0, 1.0, 0.0])
    y = np.array([1.0, 1.0, 0.0, 0.0])
    p = np.full(4, 0.5)
    mu = np.full(4, 0.5)
    ref = E.aipw_point(w, y, p, mu, mu, "reference")
    tb = E.aipw_point(w, y, p, mu, mu, "textbook")
    assert ref == pytest.approx(0.0) and tb == pytest.approx(0.0)
    y = np.array([1.0, 0.0, 1.0, 0.0])
    assert E.aipw_point(w, y, p, mu, mu, "reference") == pytest.approx(0.0)
    assert E.aipw_point(w, y, p, mu, mu, "textbook") == pytest.approx(1.0)


def test_clip_propensity():
    p = np.array([0.0, 0.2, 1.0, 0.7])
    assert list(E.clip_propensity(p)) == [0.2, 0.2, 0.7, 0.7]


def test_belloni_index_shift_quirk():
    # Q12/Q13: positive-only, union order, -1 shift, index 0 dropped
    bw = np.array([0.5, 0.0, -1.0, 0.3])
    by = np.array([0.0, 0.2, 0.0, 0.1])
    sw = np.flatnonzero(bw > 0) + 1
    sy = np.flatnonzero(by > 0) + 1
    union = []
    for v in np.concatenate([sw, sy]):
        if v not in union:
            union.append(int(v))
    assert union == [1, 4, 2]
    cols = [v - 2 for v in union if v - 1 >= 1]
    assert cols == [2, 0]


def test_dml_from_residuals_closed_form():
    rs = np.random.RandomState(5)
    wr = rs.randn(1000)
    yr = 0.7 * wr + rs.randn(1000)
    r = E.dml_from_residuals(yr, wr, "x")
    theta = wr @ yr / (wr @ wr)
    assert r.ate == pytest.approx(theta)
    psi = (yr - theta * wr) * wr
    assert r.se == pytest.approx(np.sqrt(np.mean(psi ** 2) / np.mean(wr ** 2) ** 2 / 1000))


def test_tutorial_reference_runs(tutorial):
    d, m, drop = tutorial
    assert len(drop) > 0.6 * d.n
    oracle = E.naive(d.Y, d.W, "oracle")
    naive = E.naive(m.Y, m.W)
    ols = E.ols(m.Y, m.W, m.X)
    assert 0.03 < oracle.ate < 0.16
    assert naive.ate < oracle.ate      # selection bias pushes naive down
    assert ols.ate > naive.ate
