"""Float64 CPU reference (T-ref) of every estimator in ``ate_functions.R``.

This is the parity oracle for the GPU path (R is not available here; SURVEY.md
§7.4.1). Every function takes ``(Y, W, X)`` numpy arrays and returns an
:class:`~ate_replication_causalml_amd.result.AteResult`. Reference quirks
 are reproduced under ``compat="reference"`` (default);
``compat="textbook"`` gives the intended estimator.
"""
from __future__ import annotations

import numpy as np

from ..parallel import rng
from ..result import AteResult
from . import glmnet as gn
from .linear import glm_logit, glm_predict, lm_fit


def _arr(a):
    return np.asarray(a, dtype=np.float64)


# ---------------------------------------------------------------- E1 naive
def naive(Y, W, method="naive"):
    """``naive_ate`` (ate_functions.R:3-21): diff in means; SE uses var/(n-1) (Q2)."""
    Y, W = _arr(Y), _arr(W)
    se2 = 0.0
    means = {}
    for g in (0.0, 1.0):
        yg = Y[W == g]
        means[g] = yg.mean()
        se2 += yg.var(ddof=1) / (len(yg) - 1)
    return AteResult.make(method, means[1.0] - means[0.0], np.sqrt(se2),
                          n1=int((W == 1).sum()), n0=int((W == 0).sum()))


# ---------------------------------------------------------------- E2 OLS
def ols(Y, W, X, method="Direct Method"):
    """``ate_condmean_ols`` (ate_functions.R:25-39): lm(Y ~ covariates + W)."""
    fit = lm_fit(np.column_stack([_arr(X), _arr(W)]), _arr(Y))
    return AteResult.make(method, fit.coef[-1], fit.se[-1], rank=fit.rank)


# ---------------------------------------------------------------- E16 / E7 propensities
def propensity_logistic(W, X):
    """glm(W ~ covariates, binomial) fitted values (ate_replication.Rmd:165-168)."""
    return glm_logit(_arr(X), _arr(W)).fitted


def propensity_lasso(W, X, seed=1991, nfolds=10, fold_stream=7):
    """``prop_score_lasso`` (ate_functions.R:133-146): binomial cv.glmnet,
    predicted response at lambda.1se (Q5)."""
    cv = gn.cv_glmnet(_arr(X), _arr(W), family="binomial", nfolds=nfolds, seed=seed,
                      fold_stream=fold_stream)
    return cv.predict(_arr(X), s="lambda.1se", type="response")


# ---------------------------------------------------------------- E3 IPW
def ipw_design(Y, W, X, p, compat="reference"):
    """Regressor matrix of the SE projection in ``prop_score_weight``.

    Reference quirk (Q25): the function's ``covariates`` formal is never
    supplied by the driver (ate_replication.Rmd:169,184), so
    ``wyp_df[,covariates]`` selects *every* column of the augmented frame
    [covariates, Y, W, p, tau_hat, ps_er] (ate_functions.R:45-50), each
    multiplied by ps_er. ``compat="textbook"`` uses the covariates only."""
    Y, W, X, p = _arr(Y), _arr(W), _arr(X), _arr(p)
    ps = W - p
    tau = (W - p) * Y / (p * (1 - p))
    if compat == "reference":
        frame = np.column_stack([X, Y, W, p, tau, ps])
    else:
        frame = X
    return frame * ps[:, None], tau


def ipw(Y, W, X, p, method="Propensity_Weighting", compat="reference"):
    """``prop_score_weight`` (ate_functions.R:44-63). SE = sqrt(mean(e^2))/sqrt(N) (Q22)."""
    d, tau = ipw_design(Y, W, X, p, compat)
    e = lm_fit(d, tau).residuals
    n = len(tau)
    return AteResult.make(method, tau.mean(), np.sqrt(np.mean(e ** 2)) / np.sqrt(n))


# ---------------------------------------------------------------- E4 PS-WLS
def ipw_wls(Y, W, p, method="Propensity_Regression"):
    """``prop_score_ols`` (ate_functions.R:67-86): WLS Y ~ W, weights W/p + (1-W)/(1-p)."""
    Y, W, p = _arr(Y), _arr(W), _arr(p)
    wts = W / p + (1 - W) / (1 - p)
    fit = lm_fit(W[:, None], Y, weights=wts)
    return AteResult.make(method, fit.coef[1], fit.se[1])


# ---------------------------------------------------------------- E5 / E6 LASSO
def lasso_single(Y, W, X, seed=1991, nfolds=10, fold_stream=5, method="Single-equation LASSO"):
    """``ate_condmean_lasso`` (ate_functions.R:89-108): W unpenalised; no SE (Q4)."""
    Xw = np.column_stack([_arr(X), _arr(W)])
    pf = np.r_[np.ones(Xw.shape[1] - 1), 0.0]
    cv = gn.cv_glmnet(Xw, _arr(Y), penalty_factor=pf, nfolds=nfolds, seed=seed,
                      fold_stream=fold_stream)
    return AteResult.make(method, cv.coef()[1][-1], None, lambda_1se=cv.lambda_1se)


def lasso_usual(Y, W, X, seed=1991, nfolds=10, fold_stream=6, method="Usual LASSO"):
    """``ate_lasso`` (ate_functions.R:111-130): W penalised; no SE (Q4)."""
    Xw = np.column_stack([_arr(X), _arr(W)])
    cv = gn.cv_glmnet(Xw, _arr(Y), nfolds=nfolds, seed=seed, fold_stream=fold_stream)
    return AteResult.make(method, cv.coef()[1][-1], None, lambda_1se=cv.lambda_1se)


# ---------------------------------------------------------------- AIPW pieces (E8/E9/E10)
def aipw_point(w, y, p, mu0, mu1, compat="reference"):
    """tau_hat as written (ate_functions.R:184-186): '+' on the control term (Q7);
    ``mean(est1, na.rm=TRUE)`` drops NaN (Q23)."""
    sign = 1.0 if compat == "reference" else -1.0
    est1 = w * (y - mu1) / p + sign * (1 - w) * (y - mu0) / (1 - p)
    est2 = mu1 - mu0
    return np.nanmean(est1) + np.mean(est2)


def aipw_sandwich_se(w, y, p, mu0, mu1, tau):
    """Sandwich SE (ate_functions.R:198-199): textbook IF with '-' sign."""
    ii = (w * y) / p - mu1 * (w - p) / p - (((1 - w) * y / (1 - p)) + (mu0 * (w - p) / (1 - p))) - tau
    n = len(ii)
    return np.sqrt(np.sum(ii ** 2) * n ** -2.0)


def bootstrap_counts_matrix(n, B, seed, stream0=0):
    """(B, n) resample counts; replicate b draws rows randint(seed, P_BOOT, b, j, n)."""
    out = np.empty((B, n), dtype=np.int64)
    for b in range(B):
        out[b] = rng.bootstrap_counts(n, seed, rng.P_BOOT, stream0 + b)
    return out


def aipw_bootstrap(w, y, p, mu0, mu1, B=1000, seed=1991, compat="reference"):
    """E10 ``tau_hat_dr_est`` x B (ate_functions.R:188-195, 267-283): resample the
    FIXED nuisance predictions (no refit, Q21); SE = sd(tau_b) (n-1)."""
    sign = 1.0 if compat == "reference" else -1.0
    est1 = w * (y - mu1) / p + sign * (1 - w) * (y - mu0) / (1 - p)
    est2 = mu1 - mu0
    ok = ~np.isnan(est1)
    e1 = np.where(ok, est1, 0.0)
    n = len(w)
    taus = np.empty(B)
    for b in range(B):
        c = rng.bootstrap_counts(n, seed, rng.P_BOOT, b).astype(np.float64)
        taus[b] = (c @ e1) / (c @ ok) + (c @ est2) / n
    return float(np.std(taus, ddof=1)), taus


def _aipw_result(method, w, y, p, mu0, mu1, bootstrap_se, B, seed, compat, **diag):
    tau = aipw_point(w, y, p, mu0, mu1, compat)
    if bootstrap_se:
        se, _ = aipw_bootstrap(w, y, p, mu0, mu1, B=B, seed=seed, compat=compat)
    else:
        se = aipw_sandwich_se(w, y, p, mu0, mu1, tau)
    return AteResult.make(method, tau, se, **diag)


def outcome_logit_mu(Y, W, X, counterfactual_quirk):
    """Outcome GLM Y ~ covariates + W (Q24) and mu1/mu0 predictions.
    ``counterfactual_quirk`` (Q6): ``mutate_("W = 1")`` adds a column named
    "W = 1" and leaves W untouched, so mu1 = mu0 = mu(x, W_observed)."""
    X, W, Y = _arr(X), _arr(W), _arr(Y)
    fit = glm_logit(np.column_stack([X, W]), Y)
    if counterfactual_quirk:
        mu = glm_predict(fit, np.column_stack([X, W]))
        return mu, mu.copy()
    mu1 = glm_predict(fit, np.column_stack([X, np.ones_like(W)]))
    mu0 = glm_predict(fit, np.column_stack([X, np.zeros_like(W)]))
    return mu0, mu1


def clip_propensity(p):
    """ate_functions.R:181-182: exact 0 -> min positive, exact 1 -> max below 1."""
    p = p.copy()
    pos = p[p > 0]
    below = p[p < 1]
    if pos.size:
        p = np.where(p == 0, pos.min(), p)
    if below.size:
        p = np.where(p == 1, below.max(), p)
    return p


def aipw_glm(Y, W, X, bootstrap_se=False, B=1000, seed=1991, compat="reference",
             method="Doubly Robust with logistic regression PS"):
    """``doubly_robust_glm`` (ate_functions.R:211-264): logistic outcome and
    propensity models, no clipping (Q9)."""
    Y, W, X = _arr(Y), _arr(W), _arr(X)
    mu0, mu1 = outcome_logit_mu(Y, W, X, counterfactual_quirk=False)
    p = propensity_logistic(W, X)
    return _aipw_result(method, W, Y, p, mu0, mu1, bootstrap_se, B, seed, compat)


def aipw_rf(Y, W, X, num_trees=100, bootstrap_se=False, B=1000, seed=1991, forest_seed=12325,
            compat="reference", method="Doubly Robust with Random Forest PS", splits="auto"):
    """``doubly_robust`` (ate_functions.R:149-207): logistic outcome model,
    random-forest OOB propensity (clipped, Q9), counterfactual quirk Q6 under
    ``compat="reference"``. ``splits``: models/forest.resolve_splits."""
    from ..models.forest import resolve_splits
    from .forest import rf_classifier_fit
    Y, W, X = _arr(Y), _arr(W), _arr(X)
    mu0, mu1 = outcome_logit_mu(Y, W, X, counterfactual_quirk=(compat == "reference"))
    rf = rf_classifier_fit(X, W, num_trees=num_trees, seed=forest_seed,
                           splits=resolve_splits(splits, len(Y), X.shape[1]))
    p = clip_propensity(rf.oob_proba())
    return _aipw_result(method, W, Y, p, mu0, mu1, bootstrap_se, B, seed, compat,
                        n_oob_nan=int(np.isnan(rf.oob_proba()).sum()))


# ---------------------------------------------------------------- E11 Belloni
def interaction_expand(X):
    """All ordered pairwise products incl. squares (ate_functions.R:289-296, Q10)."""
    X = _arr(X)
    n, p = X.shape
    prods = (X[:, :, None] * X[:, None, :]).reshape(n, p * p)
    return np.column_stack([X, prods])


def lambda_interp(lambdas, s):
    """glmnet's ``lambda.interp`` (linear interpolation in lambda)."""
    lam = np.asarray(lambdas, float)
    k = len(lam)
    if k == 1:
        return 0, 0, 1.0
    sfrac = (lam[0] - s) / (lam[0] - lam[k - 1])
    ln = (lam[0] - lam) / (lam[0] - lam[k - 1])
    sfrac = min(max(sfrac, ln.min()), ln.max())
    coord = np.interp(sfrac, ln, np.arange(k))
    left, right = int(np.floor(coord)), int(np.ceil(coord))
    if left == right or abs(ln[left] - ln[right]) < np.finfo(float).eps:
        return left, right, 1.0
    frac = (sfrac - ln[right]) / (ln[left] - ln[right])
    return left, right, float(frac)


def coef_at(path, s):
    left, right, frac = lambda_interp(path.lambdas, s)
    a0 = path.a0[left] * frac + path.a0[right] * (1 - frac)
    b = path.beta[left] * frac + path.beta[right] * (1 - frac)
    return a0, b


def belloni_select(Xint, W, Y, seed=1991, nfolds=10, compat="reference"):
    cw = gn.cv_glmnet(Xint, W, nfolds=nfolds, seed=seed, fold_stream=8)
    cy = gn.cv_glmnet(Xint, Y, nfolds=nfolds, seed=seed, fold_stream=9)
    s = cw.lambda_min
    _, bw = coef_at(cw.fit, s)
    _, by = coef_at(cy.fit, s if compat == "reference" else cy.lambda_min)   # Q11
    if compat == "reference":
        sw = np.flatnonzero(bw > 0) + 1                     # 1-based, positive only (Q12)
        sy = np.flatnonzero(by > 0) + 1
        union = []
        for v in np.concatenate([sw, sy]):
            if v not in union:
                union.append(int(v))
        shifted = [v - 1 for v in union]                    # Q13: '- 1' shift
        cols = [v - 1 for v in shifted if v >= 1]           # R drops index 0; to 0-based
    else:
        cols = sorted(set(np.flatnonzero(bw != 0)) | set(np.flatnonzero(by != 0)))
    return cols, cw, cy


def belloni(Y, W, X, seed=1991, nfolds=10, compat="reference", method="Belloni et.al"):
    """``belloni`` (ate_functions.R:286-328): post-double-selection on 462 features."""
    Y, W = _arr(Y), _arr(W)
    Xint = interaction_expand(X)
    cols, cw, cy = belloni_select(Xint, W, Y, seed, nfolds, compat)
    fit = lm_fit(np.column_stack([Xint[:, cols], W]), Y)
    return AteResult.make(method, fit.coef[-1], fit.se[-1], n_selected=len(cols),
                          rank=fit.rank)


# ---------------------------------------------------------------- E12/E13 DML (compat)
def chernozhukov(Y, W, X, idx1, idx2, num_trees, seed=123, splits="auto"):
    """One DML half (ate_functions.R:332-369, Q14/Q15); bins from all rows."""
    from ..models import forest as F
    Y, W, X = _arr(Y), _arr(W), _arr(X)
    splits = F.resolve_splits(splits, len(Y), X.shape[1])
    edges = F.exact_bins(X) if splits == "exact" else F.bin_edges(X)
    rf1 = F.fit_forest(X[idx1], F.KIND_CLASS, y=W[idx1], ntree=num_trees, seed=seed,
                       backend="cpu", edges=edges, splits=splits)
    rf2 = F.fit_forest(X[idx2], F.KIND_CLASS, y=Y[idx2], ntree=num_trees, seed=seed + 1,
                       backend="cpu", edges=edges, splits=splits)
    ew = rf1.predict_proba(X)
    ey = rf2.predict_proba(X)
    return resid_on_resid(Y - ey, W - ew)


def resid_on_resid(yr, wr):
    """lm(Y_resid ~ 0 + W_resid): tau, classical SE."""
    sww = wr @ wr
    tau = (wr @ yr) / sww
    rss = np.sum((yr - tau * wr) ** 2)
    se = np.sqrt(rss / (len(yr) - 1) / sww)
    return tau, se


def double_ml(Y, W, X, num_trees=100, seed=123, method="Double Machine Learning",
              splits="auto"):
    """``double_ml`` (ate_functions.R:372-389): positional 2-way split, average tau and SE."""
    n = len(Y)
    h = n // 2
    idx1, idx2 = np.arange(h), np.arange(h, n)
    t1, s1 = chernozhukov(Y, W, X, idx1, idx2, num_trees, seed, splits)
    t2, s2 = chernozhukov(Y, W, X, idx2, idx1, num_trees, seed + 2, splits)
    return AteResult.make(method, (t1 + t2) / 2, (s1 + s2) / 2)


# ---------------------------------------------------------------- E15 causal forest
def causal_forest_ate(Y, W, X, num_trees=2000, seed=12345, method="Causal Forest(GRF)",
                      nuisance_trees=None):
    """grf causal forest + AIPW ATE (ate_replication.Rmd:250-272) on the host engine."""
    from ..models import forest as F
    cf = F.causal_forest(_arr(X), _arr(Y), _arr(W), num_trees=num_trees, seed=seed,
                         nuisance_trees=nuisance_trees, backend="cpu")
    est, se = F.average_treatment_effect(cf)
    return AteResult.make(method, est, se, ate_bad=float(np.nanmean(cf.tau_oob)),
                          se_bad=float(np.sqrt(np.nanmean(cf.var_oob))))


# ---------------------------------------------------------------- K-fold DML (north star)
def dml_plr_lasso(Y, W, X, folds=5, seed=1991, lambda_rule="min",
                  method="DML cross-fit (LASSO)", fold_ids=None):
    """Partially-linear DML with K-fold cross-fitting and CV-LASSO nuisances.

    For held-out fold k the nuisances E[Y|X], E[W|X] are gaussian LASSO fits on
    the other K-1 folds, with lambda chosen by (K-1)-fold CV over those same
    folds (so every Gram the GPU needs is a sum of per-fold Grams). ``fold_ids``:
    an explicit fold of every row (default: the Philox assignment)."""
    Y, W, X = _arr(Y), _arr(W), _arr(X)
    fid = rng.fold_ids(len(Y), folds, seed, stream=0) if fold_ids is None else \
        np.asarray(fold_ids, dtype=np.int64)
    yr = np.empty_like(Y)
    wr = np.empty_like(W)
    for k in range(folds):
        tr = fid != k
        te = ~tr
        inner = fid[tr]
        inner = np.where(inner > k, inner - 1, inner)
        for target, out in ((Y, yr), (W, wr)):
            cv = gn.cv_glmnet(X[tr], target[tr], foldid=inner)
            s = "lambda.min" if lambda_rule == "min" else "lambda.1se"
            out[te] = target[te] - cv.predict(X[te], s=s)
    return dml_from_residuals(yr, wr, method)


def dml_plr_lasso_repeated(Y, W, X, folds=5, repeats=3, seed=1991, lambda_rule="min",
                           aggregate="median", method="DML cross-fit (LASSO, repeated)"):
    """Repeated cross-fitting (Chernozhukov et al. 2018 §3.4, median method): S = repeats
    K-fold partitions built from K*K micro-groups (group m = K a + b of a balanced Philox
    assignment; partition s puts it in fold (a + s b) mod K), one DML fit per partition,
    theta = median(theta_s), SE^2 = median(SE_s^2 + (theta_s - theta)^2) ("mean": means)."""
    Y, W, X = _arr(Y), _arr(W), _arr(X)
    micro = rng.fold_ids(len(Y), folds * folds, seed, stream=0)
    a, b = np.divmod(micro, folds)
    th, se = [], []
    for s in range(repeats):
        r = dml_plr_lasso(Y, W, X, folds, seed, lambda_rule, method, fold_ids=(a + s * b) % folds)
        th.append(r.ate)
        se.append(r.se)
    th, se = np.array(th), np.array(se)
    agg = np.median if aggregate == "median" else np.mean
    t = float(agg(th))
    return AteResult.make(method, t, float(np.sqrt(agg(se * se + (th - t) ** 2))),
                          n=len(Y), repeats=repeats, splits=np.stack([th, se], 1).tolist())


def dml_from_residuals(yr, wr, method):
    """Orthogonal-score combine: theta = sum(wr yr)/sum(wr^2); SE from the
    Neyman score psi = (yr - theta wr) wr, J = mean(wr^2)."""
    n = len(yr)
    j = np.mean(wr * wr)
    theta = np.mean(wr * yr) / j
    psi = (yr - theta * wr) * wr
    se = np.sqrt(np.mean(psi * psi) / (j * j) / n)
    return AteResult.make(method, theta, se, n=n)
