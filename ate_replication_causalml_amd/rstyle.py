"""R-compatible entry points: the reference's function names and calling convention
(``dataset`` data frame + column names, returning a one-row
``data.frame(Method, ATE, lower_ci, upper_ci)``), so driver code ports line by line.

Each maps onto ``api`` (see its docstring for the name table). ``covariates``
defaults to every column except the treatment and outcome, as the reference's
global ``covariates`` vector (ate_replication.Rmd:57) does for its data frame.
"""
from __future__ import annotations

import numpy as np

from . import api
from .config import BalanceConfig, RunConfig


def _split(dataset, treatment_var, outcome_var, covariates=None):
    cov = list(covariates) if covariates is not None else \
        [c for c in dataset.columns if c not in (treatment_var, outcome_var)]
    X = dataset[cov].to_numpy(dtype=np.float64)
    W = dataset[treatment_var].to_numpy(dtype=np.float64)
    Y = dataset[outcome_var].to_numpy(dtype=np.float64) if outcome_var else None
    return Y, W, X


def _df(r):
    import pandas as pd
    return pd.DataFrame([{"Method": r.method, "ATE": r.ate, "lower_ci": r.lower_ci,
                          "upper_ci": r.upper_ci}])


def _compat(run):
    return (run or RunConfig()).compat


def naive_ate(dataset, treatment_var, outcome_var, method="naive", run=None):
    """Q1: the reference groups by ``treatment_var`` but then reads the group means
    through the hard-coded column ``mean_df$W`` (ate_functions.R:11-12); with any other
    treatment name R builds ``data.frame(ATE = numeric(0), ...)`` and stops with
    "arguments imply differing number of rows". ``compat="reference"`` raises the same
    way; ``"textbook"`` uses ``treatment_var``."""
    if treatment_var != "W" and _compat(run) == "reference":
        raise ValueError("naive_ate: arguments imply differing number of rows: 1, 0 "
                         "(the reference reads mean_df$W; treatment_var must be 'W')")
    Y, W, _ = _split(dataset, treatment_var, outcome_var)
    return _df(api.ate_naive(Y, W, method=method, run=run))


def ate_condmean_ols(dataset, treatment_var, outcome_var, method="Direct Method",
                     covariates=None, run=None):
    return _df(api.ate_ols(*_split(dataset, treatment_var, outcome_var, covariates), method=method,
                           run=run))


def prop_score_weight(dataset, p, treatment_var, outcome_var, method="Propensity_Weighting",
                      covariates=None, run=None):
    Y, W, X = _split(dataset, treatment_var, outcome_var, covariates)
    return _df(api.ate_ipw(Y, W, X, np.asarray(p, dtype=np.float64), method=method, run=run))


def prop_score_ols(dataset, p, treatment_var, outcome_var, method="Propensity_Regression",
                   run=None):
    Y, W, _ = _split(dataset, treatment_var, outcome_var)
    return _df(api.ate_ipw_wls(Y, W, np.asarray(p, dtype=np.float64), method=method, run=run))


def ate_condmean_lasso(dataset, treatment_var, outcome_var, method="Single-equation LASSO",
                       covariates=None, run=None):
    return _df(api.ate_lasso_single(*_split(dataset, treatment_var, outcome_var, covariates),
                                    method=method, run=run))


def ate_lasso(dataset, treatment_var, outcome_var, method="Usual LASSO", covariates=None,
              run=None):
    return _df(api.ate_lasso(*_split(dataset, treatment_var, outcome_var, covariates),
                             method=method, run=run))


def prop_score_lasso(dataset, treatment_var, covariates=None, run=None):
    """Returns the (n, 1) matrix of predicted propensities (R: ``p_lasso[,1]``)."""
    cov = list(covariates) if covariates is not None else \
        [c for c in dataset.columns if c not in (treatment_var, "Y")]
    X = dataset[cov].to_numpy(dtype=np.float64)
    W = dataset[treatment_var].to_numpy(dtype=np.float64)
    return api.propensity_lasso(W, X, run=run)[:, None]


def doubly_robust(dataset, treatment_var, outcome_var, num_trees=100, bootstrap_se=False,
                  method="Doubly Robust with Random Forest PS", covariates=None, run=None,
                  **_swallowed):
    """``**_swallowed``: like randomForest's ``...`` (Q8), extra arguments such as
    ``seed=`` / ``type=`` are accepted and have no effect."""
    return _df(api.ate_aipw_rf(*_split(dataset, treatment_var, outcome_var, covariates),
                               num_trees=num_trees, bootstrap_se=bootstrap_se, method=method,
                               run=run))


def doubly_robust_glm(dataset, treatment_var, outcome_var, bootstrap_se=False,
                      method="Doubly Robust with logistic regression PS", covariates=None,
                      run=None):
    return _df(api.ate_aipw_glm(*_split(dataset, treatment_var, outcome_var, covariates),
                                bootstrap_se=bootstrap_se, method=method, run=run))


def belloni(dataset, treatment_var, outcome_var, method="Belloni et.al", covariates=None,
            run=None):
    return _df(api.ate_belloni(*_split(dataset, treatment_var, outcome_var, covariates),
                               method=method, run=run))


def double_ml(dataset, treatment_var, outcome_var, num_trees=100,
              method="Double Machine Learning", covariates=None, run=None, **kw):
    # the driver passes num_tree= (R partial matching, ate_replication.Rmd:232, Q19);
    # anything else is swallowed like randomForest's `...` (Q8)
    num_trees = kw.pop("num_tree", num_trees)
    return _df(api.ate_double_ml(*_split(dataset, treatment_var, outcome_var, covariates),
                                 num_trees=num_trees, method=method, run=run))


def residual_balance_ATE(dataset, treatment_var, outcome_var, optimizer="quadprog",
                         method="residual_balancing", covariates=None, run=None, df_mod=None):
    """``optimizer`` is accepted for compatibility; the QP is solved exactly by the IPM.

    Q16/Q20 (ate_functions.R:394-400, ate_replication.Rmd:240): the reference reads the
    GLOBAL ``df_mod`` and ignores ``dataset`` (the driver even passes an undefined
    symbol, harmless under lazy evaluation) and always labels the row
    "residual_balancing", ignoring ``method``. Under ``compat="reference"`` a given
    ``df_mod`` replaces ``dataset`` (which may then be None) and the label is fixed;
    ``"textbook"`` uses ``dataset`` and ``method``."""
    ref = _compat(run) == "reference"
    data = df_mod if (ref and df_mod is not None) else dataset
    label = "residual_balancing" if ref else method
    return _df(api.ate_residual_balance(*_split(data, treatment_var, outcome_var, covariates),
                                        BalanceConfig(), method=label, run=run))


def causal_forest_ate(dataset, treatment_var, outcome_var, num_trees=2000, seed=12345,
                      covariates=None, run=None):
    return _df(api.ate_causal_forest(*_split(dataset, treatment_var, outcome_var, covariates),
                                     num_trees=num_trees, seed=seed, run=run))


__all__ = ["naive_ate", "ate_condmean_ols", "prop_score_weight", "prop_score_ols",
           "ate_condmean_lasso", "ate_lasso", "prop_score_lasso", "doubly_robust",
           "doubly_robust_glm", "belloni", "double_ml", "residual_balance_ATE",
           "causal_forest_ate", "RunConfig"]


def tau_hat_dr_est(w, y, p, tauhat0x, tauhat1x, b=0, seed=1991, compat="reference"):
    """E10 helper ``tau_hat_dr_est`` (ate_functions.R:267-283): ONE with-replacement
    resample of the fixed AIPW inputs, ``mean(est1, na.rm=TRUE) + mean(est2)``. R's
    ``sample()`` is replaced by counter-based Philox draws: replicate ``b`` of ``seed``
    is the b-th of the replicates ``doubly_robust(..., bootstrap_se=TRUE)`` uses (K20)."""
    from .ops import stats as S
    import torch
    arr = [torch.as_tensor(np.asarray(v, dtype=np.float64)) for v in (w, y, p, tauhat0x,
                                                                       tauhat1x)]
    w_, y_, p_, m0, m1 = arr
    e1, e2 = S.aipw_terms(w_, y_, p_, m0, m1, compat)
    return float(S.bootstrap_multinomial(e1.contiguous(), e2.contiguous(), 1, seed, b0=b)[0])


def chernozhukov(dataset, treatment_var, outcome_var, idx1, idx2, num_trees, seed=123,
                 covariates=None, run=None):
    """E12 helper ``chernozhukov`` (ate_functions.R:332-369): RF for W trained on rows
    ``idx1``, RF for Y on ``idx2`` (0-based row positions), both predicted on all rows,
    no-intercept regression of the residuals. Returns R's ``list(tau_hat, se_hat)`` as a
    dict."""
    from .estimators import forest as DF
    Y, W, X = _split(dataset, treatment_var, outcome_var, covariates)
    dev = None if run is None or run.backend != "cpu" else "cpu"
    tau, se = DF.chernozhukov(Y, W, X, np.asarray(idx1), np.asarray(idx2), num_trees, seed,
                              device=dev)
    return {"tau_hat": float(tau), "se_hat": float(se)}
