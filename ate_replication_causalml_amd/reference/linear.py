"""Float64 reference for ``stats::lm`` / ``summary.lm`` and ``stats::glm(binomial)``.

Mirrors the semantics the reference relies on:

* ``lm`` (``ate_functions.R:28,53,74,320,363``): least squares via QR with
  LINPACK ``dqrdc2``-style limited pivoting: a column whose norm after
  projecting out the previously accepted columns falls below ``tol`` (1e-7)
  times its original norm is *aliased* (coefficient ``NA``) and moved out of
  the fit. ``summary.lm`` SE = sqrt(sigma^2 diag((X'X)^-1)), sigma^2 =
  RSS / (n - rank). Weighted fits (``weights=``, ``ate_functions.R:75``) use
  sqrt(w) scaling; sigma^2 = sum(w e^2)/(n - rank).
* ``glm(family=binomial)`` (``ate_functions.R:156,218,231``,
  ``ate_replication.Rmd:167``): IRLS as ``glm.fit`` with ``mustart=(y+0.5)/2``,
  ``epsilon=1e-8``, ``maxit=25``.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

LM_TOL = 1e-7


@dataclass
class LmFit:
    coef: np.ndarray        # NaN for aliased columns
    se: np.ndarray          # NaN for aliased columns
    aliased: np.ndarray     # bool
    rank: int
    df_resid: int
    sigma2: float
    residuals: np.ndarray
    fitted: np.ndarray


def _pivot_rank(A: np.ndarray, tol: float):
    """Sequential (column-order) rank detection equivalent to dqrdc2's limited
    pivoting. |R_jj| of an unpivoted Householder QR is the norm of column j
    after projecting out all earlier columns, so column j is aliased iff
    |R_jj| < tol * ||a_j||; aliased columns add nothing to the span, so the
    test on later columns is unchanged by dropping them."""
    norms = np.linalg.norm(A, axis=0)
    R = np.linalg.qr(A, mode="r")
    d = np.abs(np.diag(R))
    keep = np.flatnonzero((norms > 0) & (d >= tol * norms))
    return keep.astype(np.int64)


def lm_fit(X: np.ndarray, y: np.ndarray, weights=None, intercept: bool = True,
           tol: float = LM_TOL) -> LmFit:
    """``lm(y ~ X)`` (with intercept column prepended when ``intercept``)."""
    X = np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X[:, None]
    y = np.asarray(y, dtype=np.float64)
    n = X.shape[0]
    A = np.column_stack([np.ones(n), X]) if intercept else X
    sw = np.ones(n) if weights is None else np.sqrt(np.asarray(weights, dtype=np.float64))
    Aw = A * sw[:, None]
    yw = y * sw
    keep = _pivot_rank(Aw, tol)
    p = A.shape[1]
    coef = np.full(p, np.nan)
    se = np.full(p, np.nan)
    Ak = Aw[:, keep]
    beta, *_ = np.linalg.lstsq(Ak, yw, rcond=None)
    coef[keep] = beta
    fitted = A[:, keep] @ beta
    resid = y - fitted
    rank = len(keep)
    df = n - rank
    rss = float(np.sum((resid * sw) ** 2))
    sigma2 = rss / df if df > 0 else np.nan
    R = np.linalg.qr(Ak, mode="r")
    Rinv = np.linalg.solve(R, np.eye(rank))
    se[keep] = np.sqrt(sigma2 * np.sum(Rinv ** 2, axis=1))
    aliased = np.ones(p, dtype=bool)
    aliased[keep] = False
    return LmFit(coef, se, aliased, rank, df, sigma2, resid, fitted)


@dataclass
class GlmFit:
    coef: np.ndarray
    fitted: np.ndarray     # mu
    eta: np.ndarray
    deviance: float
    iters: int
    converged: bool


def _binom_dev(y, mu):
    with np.errstate(divide="ignore", invalid="ignore"):
        t1 = np.where(y > 0, y * np.log(np.where(y > 0, y / mu, 1.0)), 0.0)
        t2 = np.where(y < 1, (1 - y) * np.log(np.where(y < 1, (1 - y) / (1 - mu), 1.0)), 0.0)
    return 2.0 * np.sum(t1 + t2)


def glm_logit(X: np.ndarray, y: np.ndarray, intercept: bool = True, epsilon: float = 1e-8,
              maxit: int = 25) -> GlmFit:
    """``glm(y ~ X, family=binomial("logit"))`` via IRLS as in ``glm.fit``."""
    X = np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X[:, None]
    y = np.asarray(y, dtype=np.float64)
    n = X.shape[0]
    A = np.column_stack([np.ones(n), X]) if intercept else X
    mu = (y + 0.5) / 2.0
    eta = np.log(mu / (1 - mu))
    dev_old = _binom_dev(y, mu)
    coef = np.zeros(A.shape[1])
    converged = False
    it = 0
    for it in range(1, maxit + 1):
        mu_eta = mu * (1 - mu)
        z = eta + (y - mu) / mu_eta
        w = mu_eta
        fit = lm_fit(A, z, weights=w, intercept=False)
        coef = np.where(np.isnan(fit.coef), 0.0, fit.coef)
        eta = A @ coef
        mu = 1.0 / (1.0 + np.exp(-eta))
        mu = np.clip(mu, np.finfo(float).eps * 10, 1 - np.finfo(float).eps * 10)
        dev = _binom_dev(y, mu)
        if abs(dev - dev_old) / (abs(dev) + 0.1) < epsilon:
            converged = True
            break
        dev_old = dev
    return GlmFit(coef, mu, eta, dev, it, converged)


def glm_predict(fit: GlmFit, X: np.ndarray, intercept: bool = True) -> np.ndarray:
    X = np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X[:, None]
    A = np.column_stack([np.ones(X.shape[0]), X]) if intercept else X
    return 1.0 / (1.0 + np.exp(-(A @ fit.coef)))
