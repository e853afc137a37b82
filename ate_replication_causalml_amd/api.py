"""Public API: one function per reference estimator, each taking
``(Y, W, X, ...)`` arrays and returning an :class:`AteResult`, plus ``replicate()``
which runs the driver ``ate_replication.Rmd`` end to end (14 rows, same labels).

``run=RunConfig(backend=...)`` selects the execution path:

* ``"gpu"``  — hand-written gfx950 kernels (libatehip.so), the default when a GPU
  is visible;
* ``"cpu"``  — the same device orchestration on host tensors (CPU Gram / solver
  fallbacks, host C++ forest engine);
* ``"reference"`` — the float64 numpy T-ref (reference/), the parity oracle.

Reference function -> API name:
naive_ate -> ate_naive; ate_condmean_ols -> ate_ols; prop_score_weight -> ate_ipw;
prop_score_ols -> ate_ipw_wls; ate_condmean_lasso -> ate_lasso_single; ate_lasso ->
ate_lasso; prop_score_lasso -> propensity_lasso; doubly_robust -> ate_aipw_rf;
doubly_robust_glm -> ate_aipw_glm; belloni -> ate_belloni; double_ml ->
ate_double_ml; residual_balance_ATE -> ate_residual_balance; grf::causal_forest +
estimate_average_effect -> ate_causal_forest; K-fold DML-PLR -> ate_dml.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import numpy as np

from .config import METHODS, BalanceConfig, ReplicateConfig, RunConfig
from .result import AteResult, format_table, results_frame
from .utils import guards
from .utils.tracing import trace


def _run(run):
    return run if run is not None else RunConfig()


def _ref(run):
    return run.backend == "reference"


def _np(a):
    import torch
    if isinstance(a, torch.Tensor):
        return a.detach().double().cpu().numpy()
    return np.asarray(a, dtype=np.float64)


# ------------------------------------------------------------------ estimators
def ate_naive(Y, W, method="naive", run=None) -> AteResult:
    """E1 naive_ate (ate_functions.R:3-21)."""
    run = _run(run)
    with trace(f"ate_naive[{method}]"):
        if _ref(run):
            from .reference import estimators as R
            return R.naive(Y, W, method)
        from .estimators import linear as D
        return D.naive(Y, W, method, device=run.device())


def ate_ols(Y, W, X, method="Direct Method", run=None) -> AteResult:
    """E2 ate_condmean_ols (ate_functions.R:25-39)."""
    run = _run(run)
    with trace("ate_ols"):
        if _ref(run):
            from .reference import estimators as R
            return R.ols(Y, W, X, method)
        from .estimators import linear as D
        return D.ols(Y, W, X, method, device=run.device(), dtype=run.dtype)


def propensity_logistic(W, X, run=None) -> np.ndarray:
    """E16 glm(W ~ covariates, binomial) fitted values (ate_replication.Rmd:165-168)."""
    run = _run(run)
    with trace("propensity_logistic"):
        if _ref(run):
            from .reference import estimators as R
            return R.propensity_logistic(W, X)
        from .estimators import linear as D
        return _np(D.propensity_logistic(W, X, device=run.device(), dtype=run.dtype))


def propensity_lasso(W, X, nfolds=10, run=None) -> np.ndarray:
    """E7 prop_score_lasso (ate_functions.R:133-146): binomial cv.glmnet, lambda.1se."""
    run = _run(run)
    with trace("propensity_lasso"):
        if _ref(run):
            from .reference import estimators as R
            return R.propensity_lasso(W, X, seed=run.seed, nfolds=nfolds)
        from .estimators import linear as D
        dt = "f64" if run.dtype == "bf16" else run.dtype
        return _np(D.propensity_lasso(W, X, seed=run.seed, nfolds=nfolds, device=run.device(),
                                      dtype=dt))


def ate_ipw(Y, W, X, p, method="Propensity_Weighting", run=None) -> AteResult:
    """E3 prop_score_weight (ate_functions.R:44-63)."""
    run = _run(run)
    with trace(f"ate_ipw[{method}]"):
        if _ref(run):
            from .reference import estimators as R
            r = R.ipw(Y, W, X, p, method, compat=run.compat)
        else:
            from .estimators import linear as D
            r = D.ipw(Y, W, X, p, method, compat=run.compat, device=run.device(),
                      dtype="f64" if run.dtype == "bf16" else run.dtype)
    import torch
    r.diagnostics.update(guards.overlap_report(torch.as_tensor(_np(p)), torch.as_tensor(_np(W))))
    return r


def ate_ipw_wls(Y, W, p, method="Propensity_Regression", run=None) -> AteResult:
    """E4 prop_score_ols (ate_functions.R:67-86)."""
    run = _run(run)
    with trace("ate_ipw_wls"):
        if _ref(run):
            from .reference import estimators as R
            return R.ipw_wls(Y, W, p, method)
        from .estimators import linear as D
        return D.ipw_wls(Y, W, p, method, device=run.device(),
                         dtype="f64" if run.dtype == "bf16" else run.dtype)


def ate_lasso_single(Y, W, X, nfolds=10, method="Single-equation LASSO", run=None) -> AteResult:
    """E5 ate_condmean_lasso (ate_functions.R:89-108)."""
    run = _run(run)
    with trace("ate_lasso_single"):
        if _ref(run):
            from .reference import estimators as R
            return R.lasso_single(Y, W, X, seed=run.seed, nfolds=nfolds, method=method)
        from .estimators import lasso as DL
        return DL.lasso_single(Y, W, X, seed=run.seed, nfolds=nfolds, method=method,
                               device=run.device(), dtype=run.dtype)


def ate_lasso(Y, W, X, nfolds=10, method="Usual LASSO", run=None) -> AteResult:
    """E6 ate_lasso (ate_functions.R:111-130)."""
    run = _run(run)
    with trace("ate_lasso"):
        if _ref(run):
            from .reference import estimators as R
            return R.lasso_usual(Y, W, X, seed=run.seed, nfolds=nfolds, method=method)
        from .estimators import lasso as DL
        return DL.lasso_usual(Y, W, X, seed=run.seed, nfolds=nfolds, method=method,
                              device=run.device(), dtype=run.dtype)


def ate_aipw_rf(Y, W, X, num_trees=100, bootstrap_se=False, B=1000,
                method="Doubly Robust with Random Forest PS", run=None,
                splits="auto") -> AteResult:
    """E8 doubly_robust (ate_functions.R:149-207). ``splits``: "exact" = randomForest split
    semantics (every distinct value, midpoint thresholds), "binned" = 256-bin histograms,
    "auto" = exact up to 65536 rows (the tutorial's df_mod)."""
    run = _run(run)
    with trace("ate_aipw_rf", trees=num_trees):
        if _ref(run):
            from .reference import estimators as R
            return R.aipw_rf(Y, W, X, num_trees=num_trees, bootstrap_se=bootstrap_se, B=B,
                             seed=run.seed, compat=run.compat, method=method, splits=splits)
        from .estimators import forest as DF
        return DF.aipw_rf(Y, W, X, num_trees=num_trees, bootstrap_se=bootstrap_se, B=B,
                          seed=run.seed, compat=run.compat, method=method, device=run.device(),
                          splits=splits)


def ate_aipw_glm(Y, W, X, bootstrap_se=False, B=1000,
                 method="Doubly Robust with logistic regression PS", run=None) -> AteResult:
    """E9 doubly_robust_glm (ate_functions.R:211-264)."""
    run = _run(run)
    with trace("ate_aipw_glm"):
        if _ref(run):
            from .reference import estimators as R
            return R.aipw_glm(Y, W, X, bootstrap_se=bootstrap_se, B=B, seed=run.seed,
                              compat=run.compat, method=method)
        from .estimators import linear as D
        return D.aipw_glm(Y, W, X, bootstrap_se=bootstrap_se, B=B, seed=run.seed,
                          compat=run.compat, method=method, device=run.device(),
                          dtype="f64" if run.dtype == "bf16" else run.dtype)


def ate_belloni(Y, W, X, nfolds=10, method="Belloni et.al", run=None) -> AteResult:
    """E11 belloni (ate_functions.R:286-328)."""
    run = _run(run)
    with trace("ate_belloni"):
        if _ref(run):
            from .reference import estimators as R
            return R.belloni(Y, W, X, seed=run.seed, nfolds=nfolds, compat=run.compat,
                             method=method)
        from .estimators import lasso as DL
        return DL.belloni(Y, W, X, seed=run.seed, nfolds=nfolds, compat=run.compat,
                          method=method, device=run.device(), dtype=run.dtype)


def ate_double_ml(Y, W, X, num_trees=100, method="Double Machine Learning", run=None,
                  splits="auto") -> AteResult:
    """E12/E13 double_ml (ate_functions.R:332-389): two-half RF cross-fitting; ``splits``
    as in ate_aipw_rf."""
    run = _run(run)
    with trace("ate_double_ml", trees=num_trees):
        if _ref(run):
            from .reference import estimators as R
            return R.double_ml(Y, W, X, num_trees=num_trees, method=method, splits=splits)
        from .estimators import forest as DF
        return DF.double_ml(Y, W, X, num_trees=num_trees, method=method, device=run.device(),
                            splits=splits)


def ate_dml(Y, W, X, folds=5, lambda_rule="min", method="DML cross-fit (LASSO)",
            run=None, repeats=1, aggregate="median") -> AteResult:
    """K-fold cross-fit partially linear DML with CV-LASSO nuisances (north-star).
    ``repeats`` > 1: repeated cross-fitting over that many distinct K-fold partitions
    (Chernozhukov et al. 2018 §3.4), ``aggregate`` "median" (default) or "mean"; the
    partitions share one Gram pass (estimators/lasso.dml_repeated_phases)."""
    run = _run(run)
    with trace("ate_dml", folds=folds, repeats=repeats):
        if repeats > 1:
            if _ref(run):
                from .reference import estimators as R
                return R.dml_plr_lasso_repeated(Y, W, X, folds, repeats, run.seed, lambda_rule,
                                                aggregate)
            from .estimators import lasso as DL
            return DL.dml_plr_lasso_repeated(Y, W, X, folds, repeats, run.seed, lambda_rule,
                                             aggregate, device=run.device(), dtype=run.dtype)
        if _ref(run):
            from .reference import estimators as R
            return R.dml_plr_lasso(Y, W, X, folds=folds, seed=run.seed, lambda_rule=lambda_rule,
                                   method=method)
        from .estimators import lasso as DL
        return DL.dml_plr_lasso(Y, W, X, folds=folds, seed=run.seed, lambda_rule=lambda_rule,
                                method=method, device=run.device(), dtype=run.dtype)


def ate_residual_balance(Y, W, X, balance: BalanceConfig | None = None,
                         method="residual_balancing", run=None) -> AteResult:
    """E14 residual_balance_ATE (ate_functions.R:393-405) -> balanceHD::residualBalance.ate."""
    run = _run(run)
    bc = balance or BalanceConfig()
    with trace("ate_residual_balance"):
        if _ref(run):
            from .reference.balance import residual_balance_ate
            return residual_balance_ate(Y, W, X, zeta=bc.zeta, alpha=bc.alpha, seed=run.seed,
                                        scale_x=bc.scale_x,
                                        allow_negative=bc.allow_negative_weights, method=method)
        from .estimators.balance import residual_balance
        return residual_balance(Y, W, X, zeta=bc.zeta, alpha=bc.alpha, seed=run.seed,
                                scale_x=bc.scale_x, method=method, device=run.device(),
                                dtype="f64" if run.dtype == "bf16" else run.dtype,
                                allow_negative=bc.allow_negative_weights)


def ate_causal_forest(Y, W, X, num_trees=2000, seed=12345, method="Causal Forest(GRF)",
                      run=None) -> AteResult:
    """E15 grf::causal_forest + estimate_average_effect (ate_replication.Rmd:250-272)."""
    run = _run(run)
    with trace("ate_causal_forest", trees=num_trees):
        if _ref(run):
            from .reference import estimators as R
            return R.causal_forest_ate(Y, W, X, num_trees=num_trees, seed=seed, method=method)
        from .estimators import forest as DF
        return DF.causal_forest_ate(Y, W, X, num_trees=num_trees, seed=seed, method=method,
                                    device=run.device(), compat=run.compat)


def ate_aipw_crossfit(Y, W, X, folds=5, learner="rf", num_trees=500, run=None, comm=None,
                      **kw) -> AteResult:
    """K-fold cross-fitted AIPW (textbook signs) with rf / glm / gbdt nuisances
    (BASELINE config 3); ``comm`` shards the forests' trees over ranks."""
    run = _run(run)
    with trace("ate_aipw_crossfit", learner=learner, folds=folds):
        from .estimators.crossfit import aipw_crossfit
        return aipw_crossfit(Y, W, X, folds=folds, learner=learner, num_trees=num_trees,
                             seed=run.seed, device=run.device() if not _ref(run) else "cpu",
                             comm=comm, **kw)


def ate_causal_forest_bootstrap(Y, W, X, num_trees=2000, B=1000, seed=12345, run=None,
                                comm=None) -> AteResult:
    """Causal-forest ATE with a B-replicate bootstrap SE sharded over ranks (config 4)."""
    run = _run(run)
    with trace("ate_causal_forest_bootstrap", trees=num_trees, B=B):
        from .estimators.crossfit import causal_forest_bootstrap
        return causal_forest_bootstrap(Y, W, X, num_trees=num_trees, B=B, seed=seed,
                                       boot_seed=run.seed,
                                       device=run.device() if not _ref(run) else "cpu",
                                       comm=comm, compat=run.compat)


# ------------------------------------------------------------------ driver
@dataclass
class Replication:
    results: list
    n_dropped: int
    n_mod: int
    tau_true: float
    seconds: dict = field(default_factory=dict)

    def frame(self):
        return results_frame(self.results)

    def table(self):
        return format_table(self.results)


def _result_arrays(r: AteResult) -> dict:
    import json
    return {"method": np.array(r.method), "vals": np.array([r.ate, r.se, r.lower_ci, r.upper_ci]),
            "diag": np.array(json.dumps(r.diagnostics, default=str))}


def _result_from(d: dict) -> AteResult:
    import json
    v = d["vals"]
    return AteResult(str(d["method"]), float(v[0]), float(v[1]), float(v[2]), float(v[3]),
                     json.loads(str(d["diag"])))


def replicate(data=None, config: ReplicateConfig | None = None, log_path=None, plot_path=None,
              verbose=False, checkpoint_dir=None) -> Replication:
    """ate_replication.Rmd end to end: oracle on the RCT sample, selection bias
    (pt=pc=0.85), then the 13 estimators on df_mod in the driver's order.

    ``checkpoint_dir``: every finished row is saved there (utils/checkpoint.py, keyed by
    the config and a fingerprint of the data); a rerun loads finished rows and computes
    only the missing ones — identical results, since every random draw is keyed by seed."""
    from .data.dgp import make_tutorial_data
    from .data.selection import apply_selection_bias
    cfg = config or ReplicateConfig()
    run = cfg.run
    if data is None:
        data = make_tutorial_data(cfg.n_obs, run.seed)
    mod, drop = apply_selection_bias(data, cfg.pt, cfg.pc, cfg.selection_compat)
    Y, W, X = mod.Y, mod.W, mod.X
    want = set(cfg.include) if cfg.include else set(METHODS)
    results, secs = [], {}
    ck, dkey = None, ""
    if checkpoint_dir is not None:
        from .utils.checkpoint import Checkpoint, fingerprint
        ck = Checkpoint(checkpoint_dir, cfg.to_dict())
        dkey = fingerprint(Y, W, X, data.Y, data.W)

    def add(label, fn):
        if label not in want:
            return None
        t0 = time.perf_counter()
        if ck is not None and ck.has(label, dkey):
            r = _result_from(ck.load(label, dkey))
        else:
            r = fn()
            if ck is not None:
                ck.save(label, dkey, **_result_arrays(r))
        secs[label] = time.perf_counter() - t0
        if verbose:
            print(f"{label:45s} {r.ate:9.4f}  ({secs[label]:.2f}s)", flush=True)
        results.append(r)
        return r

    add("oracle", lambda: ate_naive(data.Y, data.W, method="oracle", run=run))
    add("naive", lambda: ate_naive(Y, W, run=run))
    add("Direct Method", lambda: ate_ols(Y, W, X, run=run))
    cache = {}

    def p_log():
        if "log" not in cache:
            t0 = time.perf_counter()
            cache["log"] = propensity_logistic(W, X, run=run)
            secs["propensity_logistic"] = time.perf_counter() - t0
        return cache["log"]

    def p_las():
        if "las" not in cache:
            t0 = time.perf_counter()
            cache["las"] = propensity_lasso(W, X, run=run)
            secs["propensity_lasso"] = time.perf_counter() - t0
        return cache["las"]

    add("Propensity_Weighting", lambda: ate_ipw(Y, W, X, p_log(), run=run))
    add("Propensity_Regression", lambda: ate_ipw_wls(Y, W, p_log(), run=run))
    add("Propensity_Weighting_LASSOPS",
        lambda: ate_ipw(Y, W, X, p_las(), method="Propensity_Weighting_LASSOPS", run=run))
    add("Single-equation LASSO", lambda: ate_lasso_single(Y, W, X, run=run))
    add("Usual LASSO", lambda: ate_lasso(Y, W, X, run=run))
    add("Doubly Robust with Random Forest PS",
        lambda: ate_aipw_rf(Y, W, X, num_trees=cfg.dr_trees, bootstrap_se=cfg.bootstrap_se,
                            B=cfg.B, run=run))
    add("Doubly Robust with logistic regression PS",
        lambda: ate_aipw_glm(Y, W, X, bootstrap_se=cfg.bootstrap_se, B=cfg.B, run=run))
    add("Belloni et.al", lambda: ate_belloni(Y, W, X, run=run))
    add("Double Machine Learning", lambda: ate_double_ml(Y, W, X, num_trees=cfg.dml_trees, run=run))
    add("residual_balancing", lambda: ate_residual_balance(Y, W, X, cfg.balance, run=run))
    add("Causal Forest(GRF)",
        lambda: ate_causal_forest(Y, W, X, num_trees=cfg.cf_trees, seed=cfg.cf_seed, run=run))
    rep = Replication(results, len(drop), len(Y), data.tau_true, secs)
    if log_path:
        from .utils.logging import write_jsonl
        write_jsonl(log_path, results, backend=run.backend, n_obs=cfg.n_obs, n_mod=len(Y),
                    n_dropped=len(drop), seconds=secs)
    if plot_path:
        from .utils.logging import pointrange_plot
        pointrange_plot(results, plot_path, title="ATE by method (df_mod)")
    return rep


__all__ = [
    "ate_naive", "ate_ols", "propensity_logistic", "propensity_lasso", "ate_ipw", "ate_ipw_wls",
    "ate_lasso_single", "ate_lasso", "ate_aipw_rf", "ate_aipw_glm", "ate_belloni",
    "ate_double_ml", "ate_dml", "ate_residual_balance", "ate_causal_forest", "replicate",
    "ate_aipw_crossfit", "ate_causal_forest_bootstrap",
    "Replication", "AteResult", "RunConfig", "ReplicateConfig", "BalanceConfig",
]
