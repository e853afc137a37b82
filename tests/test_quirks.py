"""Quirk register: one test per reference quirk Q1-Q25, each
pinning the ``compat="reference"`` behaviour (and, where one exists, the
``compat="textbook"`` alternative). Reference sites are cited per test."""
import numpy as np
import pytest

from ate_replication_causalml_amd import rstyle
from ate_replication_causalml_amd.config import RunConfig
from ate_replication_causalml_amd.data.selection import drop_indices, r_round, selection_masks
from ate_replication_causalml_amd.reference import estimators as E
from ate_replication_causalml_amd.reference import glmnet as gn

REF = RunConfig(backend="reference", compat="reference")
TXT = RunConfig(backend="reference", compat="textbook")
CPU = RunConfig(backend="cpu")


@pytest.fixture(scope="module")
def small(tutorial):
    _, m, _ = tutorial
    return m


def test_q01_naive_hardcodes_W(small):
    # ate_functions.R:11-12 read mean_df$W whatever treatment_var is
    df = small.to_frame().rename(columns={"W": "T"})
    with pytest.raises(ValueError, match="differing number of rows"):
        rstyle.naive_ate(df, "T", "Y", run=REF)
    out = rstyle.naive_ate(df, "T", "Y", run=TXT)
    assert np.isfinite(out.ATE[0])


def test_q02_naive_se_var_over_n_minus_1(small):
    # ate_functions.R:9,15: y_var/(count-1), y_var itself already the (n-1) variance
    r = E.naive(small.Y, small.W)
    y1, y0 = small.Y[small.W == 1], small.Y[small.W == 0]
    want = np.sqrt(y1.var(ddof=1) / (len(y1) - 1) + y0.var(ddof=1) / (len(y0) - 1))
    assert r.se == pytest.approx(want, rel=1e-14)


def test_q03_covariates_default_to_the_frame(small):
    # ate_functions.R:91,113,135,289 read the global `covariates` = every covariate column
    df = small.to_frame()
    a = rstyle.ate_condmean_ols(df, "W", "Y", run=REF)
    b = E.ols(small.Y, small.W, small.X)
    assert a.ATE[0] == pytest.approx(b.ate, rel=1e-12)


def test_q04_lasso_rows_have_degenerate_ci(small):
    # ate_functions.R:107,129: lower_ci = upper_ci = ATE
    for f in (rstyle.ate_condmean_lasso, rstyle.ate_lasso):
        out = f(small.to_frame(), "W", "Y", run=REF)
        assert out.lower_ci[0] == out.ATE[0] == out.upper_ci[0]


def test_q05_coef_and_predict_default_to_lambda_1se(small):
    # ate_functions.R:106,128,144: coef()/predict() on cv.glmnet use s = "lambda.1se"
    cv = gn.cv_glmnet(small.X, small.W, family="binomial", nfolds=10, seed=1991, fold_stream=7)
    a0, b = cv.coef()
    a1, b1 = cv.coef("lambda.1se")
    assert a0 == a1 and np.array_equal(b, b1)
    p = E.propensity_lasso(small.W, small.X)
    assert np.allclose(p, cv.predict(small.X, s="lambda.1se"))


def test_q06_doubly_robust_counterfactual_quirk(small):
    # ate_functions.R:160,164 mutate_("W = 1") leaves W untouched -> mu1 == mu0
    mu0, mu1 = E.outcome_logit_mu(small.Y, small.W, small.X, counterfactual_quirk=True)
    assert np.array_equal(mu0, mu1)
    mu0, mu1 = E.outcome_logit_mu(small.Y, small.W, small.X, counterfactual_quirk=False)
    assert not np.allclose(mu0, mu1)


def test_q07_aipw_plus_sign_on_control_term():
    # ate_functions.R:184,241,279 '+' in the point estimate; :198,255 '-' in the IF
    w = np.array([1.0, 0.0, 1.0, 0.0])
    y = np.array([1.0, 0.0, 1.0, 0.0])
    p = np.full(4, 0.5)
    mu = np.full(4, 0.5)
    assert E.aipw_point(w, y, p, mu, mu, "reference") == pytest.approx(0.0)
    assert E.aipw_point(w, y, p, mu, mu, "textbook") == pytest.approx(1.0)
    ii_se = E.aipw_sandwich_se(w, y, p, mu, mu, 1.0)
    assert ii_se == pytest.approx(0.0)          # the IF uses '-': exact for the textbook tau


def test_q08_random_forest_seed_and_type_are_swallowed(small):
    # ate_functions.R:172-173: seed=/type= fall into randomForest's `...`
    df = small.to_frame()
    a = rstyle.doubly_robust(df, "W", "Y", 20, run=CPU)
    b = rstyle.doubly_robust(df, "W", "Y", 20, run=CPU, seed=999, type="classification")
    assert a.ATE[0] == b.ATE[0] and a.upper_ci[0] == b.upper_ci[0]


def test_q09_rf_propensity_clipped_glm_not():
    # ate_functions.R:181-182 clip exact 0/1 (RF OOB); :231-234 glm fitted, unclipped
    assert list(E.clip_propensity(np.array([0.0, 0.3, 1.0, 0.6]))) == [0.3, 0.3, 0.6, 0.6]
    inner = np.array([0.2, 0.5])
    assert np.array_equal(E.clip_propensity(inner), inner)


def test_q10_belloni_interactions_include_squares_and_both_orders():
    # ate_functions.R:290-296: 21 + 21*21 = 462 columns, x1*x2 and x2*x1 both present
    X = np.arange(6.0).reshape(2, 3) + 1
    Z = E.interaction_expand(X)
    assert Z.shape == (2, 3 + 9)
    assert np.array_equal(Z[:, 3 + 1], Z[:, 3 + 3])        # x0*x1 == x1*x0
    assert np.array_equal(Z[:, 3], X[:, 0] ** 2)            # square


def test_q11_to_q13_belloni_selection(small):
    # :309 Y-model coefficients at the W model's lambda.min; :312-313 positive only;
    # :314,317 '- 1' index shift with index 0 dropped
    Z = E.interaction_expand(small.X[:, :6])
    cols, cw, cy = E.belloni_select(Z, small.W, small.Y, compat="reference")
    _, bw = E.coef_at(cw.fit, cw.lambda_min)
    _, by = E.coef_at(cy.fit, cw.lambda_min)             # Q11: W's lambda for Y
    union = []
    for v in np.concatenate([np.flatnonzero(bw > 0) + 1, np.flatnonzero(by > 0) + 1]):
        if v not in union:
            union.append(int(v))
    want = [v - 2 for v in union if v - 1 >= 1]
    assert cols == want
    tcols, _, _ = E.belloni_select(Z, small.W, small.Y, compat="textbook")
    assert tcols == sorted(set(tcols))


def test_q14_double_ml_positional_halves_and_averaged_se(small):
    # ate_functions.R:374-383: idx1 = first floor(N/2) rows; tau and SE are both averaged
    n = len(small.Y)
    h = n // 2
    t1, s1 = E.chernozhukov(small.Y, small.W, small.X, np.arange(h), np.arange(h, n), 10, 123)
    t2, s2 = E.chernozhukov(small.Y, small.W, small.X, np.arange(h, n), np.arange(h), 10, 125)
    r = E.double_ml(small.Y, small.W, small.X, num_trees=10, seed=123)
    assert r.ate == pytest.approx((t1 + t2) / 2) and r.se == pytest.approx((s1 + s2) / 2)


def test_q15_dml_outcome_learner_is_a_classifier(small):
    # ate_functions.R:336 factor(Y): Y-hat are vote shares in [0, 1]
    from ate_replication_causalml_amd.models import forest as F
    rf = F.fit_forest(small.X, F.KIND_CLASS, y=small.Y, ntree=10, seed=1, backend="cpu")
    pr = rf.predict_proba(small.X)
    assert pr.min() >= 0 and pr.max() <= 1
    assert np.allclose(pr * 10, np.round(pr * 10))        # fractions of 10 tree votes


def test_q16_q20_residual_balance_uses_df_mod_and_fixed_label(small):
    # ate_functions.R:394-400 global df_mod, Method always "residual_balancing";
    # ate_replication.Rmd:240 passes an undefined `dataset`
    df = small.to_frame().iloc[:1500]
    a = rstyle.residual_balance_ATE(None, "W", "Y", optimizer="pogs", method="mine",
                                    df_mod=df, run=CPU)
    assert a.Method[0] == "residual_balancing"
    b = rstyle.residual_balance_ATE(df, "W", "Y", method="mine",
                                    run=RunConfig(backend="cpu", compat="textbook"))
    assert b.Method[0] == "mine" and a.ATE[0] == pytest.approx(b.ATE[0])


def test_q17_selection_rule_repeats_p2002_omits_p2004():
    # ate_replication.Rmd:104
    names = ["yob", "city", "g2000", "g2002", "p2000", "p2002", "p2004"]
    X = np.zeros((1, len(names)))
    X[0, names.index("p2004")] = 1.0                       # only p2004 set
    dt_ref, _ = selection_masks(X, names, "reference")
    dt_txt, _ = selection_masks(X, names, "textbook")
    assert not dt_ref[0] and dt_txt[0]


def test_q18_drops_first_rows_in_order():
    # ate_replication.Rmd:116-117: x[1:round(0.85 k)], not a random 85 %
    names = ["yob", "city", "g2000", "g2002", "p2000", "p2002", "p2004"]
    X = np.zeros((20, len(names)))
    X[:, names.index("g2000")] = 1.0                      # every treated row qualifies
    W = np.ones(20)
    d = drop_indices(X, W, names)
    assert list(d) == list(range(r_round(0.85 * 20)))
    assert r_round(2.5) == 2 and r_round(3.5) == 4        # R rounds half to even


def test_q19_num_tree_partial_match(small):
    # ate_replication.Rmd:232 passes num_tree= (partial match of num_trees)
    df = small.to_frame().iloc[:800]
    a = rstyle.double_ml(df, "W", "Y", num_tree=7, run=CPU)
    b = rstyle.double_ml(df, "W", "Y", num_trees=7, run=CPU)
    assert a.ATE[0] == b.ATE[0]


def test_q21_bootstrap_resamples_fixed_nuisances():
    # ate_functions.R:188-195,267-283: no refit, sd over B replicates (n-1)
    rs = np.random.RandomState(0)
    n = 50
    w = (rs.rand(n) < 0.5).astype(float)
    y = (rs.rand(n) < 0.4).astype(float)
    p = rs.uniform(0.2, 0.8, n)
    mu0, mu1 = rs.rand(n), rs.rand(n)
    se, taus = E.aipw_bootstrap(w, y, p, mu0, mu1, B=5, seed=3)
    counts = E.bootstrap_counts_matrix(n, 5, 3)
    for b in range(5):
        idx = np.repeat(np.arange(n), counts[b])
        want = E.aipw_point(w[idx], y[idx], p[idx], mu0[idx], mu1[idx])
        assert taus[b] == pytest.approx(want, rel=1e-12)
    assert se == pytest.approx(np.std(taus, ddof=1))


def test_q22_ipw_se_mean_square_no_dof(small):
    # ate_functions.R:57: sqrt(mean(e^2)) / sqrt(N)
    from ate_replication_causalml_amd.reference.linear import lm_fit
    p = E.propensity_logistic(small.W, small.X)
    r = E.ipw(small.Y, small.W, small.X, p)
    d, tau = E.ipw_design(small.Y, small.W, small.X, p)
    e = lm_fit(d, tau).residuals
    assert r.se == pytest.approx(np.sqrt(np.mean(e ** 2)) / np.sqrt(len(tau)), rel=1e-12)


def test_q23_mean_na_rm_drops_nan():
    # ate_functions.R:186 mean(est1, na.rm = TRUE)
    w = np.array([1.0, 0.0, 1.0])
    y = np.array([1.0, 0.0, 0.0])
    p = np.array([0.5, 1.0, 0.5])             # (1-w)(y-mu0)/(1-p) = 0/0 for row 2
    mu = np.zeros(3)
    t = E.aipw_point(w, y, p, mu, mu)
    assert np.isfinite(t) and t == pytest.approx(np.mean([2.0, 0.0]))


def test_q24_outcome_glm_uses_covariates_and_W(small):
    # ate_functions.R:152-153 `Y ~ .` over covariates + W
    mu0, mu1 = E.outcome_logit_mu(small.Y, small.W, small.X, counterfactual_quirk=False)
    from ate_replication_causalml_amd.reference.linear import glm_logit, glm_predict
    fit = glm_logit(np.column_stack([small.X, small.W]), small.Y)
    assert np.allclose(mu1, glm_predict(fit, np.column_stack([small.X, np.ones_like(small.W)])))


def test_q25_ipw_projection_uses_the_whole_frame(small):
    # ate_functions.R:45-50 with `covariates` unset by the driver: every frame column
    p = E.propensity_logistic(small.W, small.X)
    d, _ = E.ipw_design(small.Y, small.W, small.X, p, "reference")
    d2, _ = E.ipw_design(small.Y, small.W, small.X, p, "textbook")
    assert d.shape[1] == small.X.shape[1] + 5 and d2.shape[1] == small.X.shape[1]
