"""Float64 reference for ``glmnet`` / ``cv.glmnet``.

Call sites: ``ate_functions.R:101,123,139,304,305`` (gaussian and binomial
LASSO with 10-fold CV) and balanceHD's per-arm elastic net (E14).

Semantics reproduced from glmnet's Fortran ``elnet1`` / ``lognet`` drivers:

* covariates standardised with the (uniform) observation weights
  (population SD), y centred and scaled by its SD (gaussian);
* ``penalty.factor`` rescaled to sum to the number of variables; variables
  with factor 0 are unpenalised (E5's ``W``, ``ate_functions.R:98``);
* lambda path: 100 values, ``lambda.min.ratio`` = 1e-4 (n > p) or 1e-2,
  lambda_max = max |gradient| / penalty factor at the fit with only the
  unpenalised variables; early path stop when the deviance ratio changes by
  less than 1e-5 relative or exceeds 0.999 (after 5 lambdas);
* coordinate descent in *covariance mode* over the standardised Gram with
  the glmnet iteration structure (full pass, then active-set passes until
  ``max_j xv_j * delta_j^2 < thresh``); binomial uses an outer Newton
  (IRLS) quadratic approximation with working weights ``q(1-q)`` clamped at
  1e-5 and an unpenalised intercept coordinate; threshold scaled by the null
  deviance;
* cv.glmnet: fold-wise refits on the full-data lambda sequence, per-fold mean
  loss (MSE or binomial deviance), ``cvm`` = fold-size weighted mean,
  ``cvsd`` = sqrt(weighted var / (K-1)), ``lambda.min`` = largest lambda
  attaining min cvm, ``lambda.1se`` = largest lambda with cvm <= cvm_min +
  cvsd_min. ``coef``/``predict`` default to ``lambda.1se`` (quirk Q5).

The GPU path (``models/enet.py``) runs the same algorithm on Gram matrices
built by the MFMA kernel and is checked against this module.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from ..parallel import rng

BIG = 9.9e35
FDEV = 1e-5
DEVMAX = 0.999
MNLAM = 5
PMIN = 1e-5


@dataclass
class GlmnetPath:
    family: str
    lambdas: np.ndarray      # (L,) original scale
    a0: np.ndarray           # (L,)
    beta: np.ndarray         # (L, p) original scale
    dev_ratio: np.ndarray
    npasses: int

    def predict_link(self, X, idx=None):
        X = np.asarray(X, dtype=np.float64)
        if idx is None:
            return self.a0[None, :] + X @ self.beta.T
        return self.a0[idx] + X @ self.beta[idx]

    def predict(self, X, idx=None):
        eta = self.predict_link(X, idx)
        if self.family == "binomial":
            return 1.0 / (1.0 + np.exp(-eta))
        return eta


def _rescale_pf(pf, p):
    vp = np.maximum(np.asarray(pf, dtype=np.float64), 0.0) if pf is not None else np.ones(p)
    return vp * p / vp.sum()


def cd_solve(C, g, a, vp, xv, ab, dem, thr, ju, cint=None, gint=None, xmz=None, maxit=100000,
             state=None):
    """Covariance-mode coordinate descent at one lambda (in place on a, g).

    C: (p,p) Gram of the (standardised, working-weighted) design; g: gradient
    X'r; optional unpenalised intercept coordinate with cross terms ``cint``
    (p,), gradient ``gint`` (scalar, returned) and curvature ``xmz``.
    Structure: full pass -> (active passes until converged) -> full pass ...
    """
    p = len(g)
    active = state if state is not None else np.zeros(p, dtype=bool)
    npass = 0
    b0_delta = 0.0
    rsq_delta = 0.0

    def one_pass(idx_list):
        nonlocal gint, b0_delta, rsq_delta
        dlx = 0.0
        pos = 0
        idx_list = np.asarray(idx_list)
        while pos < len(idx_list):
            rem = idx_list[pos:]
            # next coordinate that can change: nonzero, or |g| beyond its threshold
            u_rem = g[rem] + a[rem] * xv[rem]
            cand = (a[rem] != 0) | (np.abs(u_rem) > vp[rem] * ab)
            if not cand.any():
                break
            off = int(np.argmax(cand))
            j = int(rem[off])
            pos += off + 1
            ak = a[j]
            u = g[j] + ak * xv[j]
            v = abs(u) - vp[j] * ab
            anew = np.sign(u) * v / (xv[j] + vp[j] * dem) if v > 0 else 0.0
            if anew == ak:
                continue
            active[j] = True
            d = anew - ak
            a[j] = anew
            rsq_delta += d * (2.0 * g[j] - d * xv[j])   # glmnet's incremental R^2
            dlx = max(dlx, xv[j] * d * d)
            g[:] -= C[:, j] * d
            if cint is not None:
                gint -= cint[j] * d
        if cint is not None:
            d = gint / xmz
            if d != 0.0:
                b0_delta += d
                g[:] -= cint * d
                gint -= xmz * d
                dlx = max(dlx, xmz * d * d)
        return dlx

    full = np.flatnonzero(ju)
    while npass < maxit:
        npass += 1
        dlx = one_pass(full)
        if dlx < thr:
            break
        while npass < maxit:
            npass += 1
            dlx = one_pass(np.flatnonzero(active))
            if dlx < thr:
                break
    cd_solve.last_rsq_delta = rsq_delta
    return npass, gint, b0_delta, active


def _lambda_seq_iter(nlam, flmin, ulam):
    """Yields (m, alm or None) — None means 'compute lambda_max now'."""
    for m in range(nlam):
        if ulam is not None:
            yield m, ulam[m]
        elif m == 0:
            yield m, BIG
        elif m == 1:
            yield m, None
        else:
            yield m, "alf"


def elnet_gaussian(X, y, alpha=1.0, penalty_factor=None, lambdas=None, nlambda=100,
                   lambda_min_ratio=None, thresh=1e-7, maxit=100000, weights=None):
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64).ravel()
    n, p = X.shape
    w = np.full(n, 1.0 / n) if weights is None else np.asarray(weights, float) / np.sum(weights)
    xm = w @ X
    xs = np.sqrt(np.maximum(w @ (X * X) - xm * xm, 0.0))
    ju = xs > 0
    xs_safe = np.where(ju, xs, 1.0)
    ym = w @ y
    ys = np.sqrt(w @ (y * y) - ym * ym)
    Xs = (X - xm) / xs_safe
    ysd = (y - ym) / ys
    C = (Xs * w[:, None]).T @ Xs
    g = (Xs * w[:, None]).T @ ysd
    return _elnet_core(C, g, np.ones(p), xm, xs_safe, ym, ys, ju, alpha, penalty_factor, lambdas,
                       nlambda, lambda_min_ratio if lambda_min_ratio is not None else
                       (1e-4 if n > p else 1e-2), thresh, maxit)


def _elnet_core(C, g, xv, xm, xs, ym, ys, ju, alpha, penalty_factor, lambdas, nlambda, flmin,
                thresh, maxit):
    """Gaussian path from standardised sufficient statistics (shared with the
    device path, which obtains C/g from the MFMA Gram)."""
    p = len(g)
    vp = _rescale_pf(penalty_factor, p)
    g = g.copy()
    a = np.zeros(p)
    ulam = None if lambdas is None else np.sort(np.asarray(lambdas, float))[::-1] / ys
    nlam = nlambda if ulam is None else len(ulam)
    alf = flmin ** (1.0 / (nlam - 1)) if ulam is None else 1.0
    betas, lams, devs = [], [], []
    alm = 0.0
    rsq = 0.0
    npass_tot = 0
    active = np.zeros(p, dtype=bool)
    for m, spec in _lambda_seq_iter(nlam, flmin, ulam):
        if spec is None:
            mask = ju & (vp > 0)
            alm = alf * (np.max(np.abs(g[mask]) / vp[mask]) if mask.any() else 0.0) / max(alpha, 1e-3)
        elif isinstance(spec, str):
            alm *= alf
        else:
            alm = spec
        npass, _, _, active = cd_solve(C, g, a, vp, xv, alm * alpha, alm * (1 - alpha), thresh, ju,
                                       maxit=maxit - npass_tot, state=active)
        npass_tot += npass
        rsq += cd_solve.last_rsq_delta   # 1 - RSS/TSS on the standardised scale
        betas.append(a.copy())
        lams.append(alm)
        devs.append(rsq)
        if ulam is None and m >= MNLAM - 1 and m > 0:
            if devs[-1] - devs[-2] < FDEV * devs[-1] or devs[-1] > DEVMAX:
                break
    lams = np.array(lams)
    if ulam is None and len(lams) >= 3:
        lams[0] = np.exp(2 * np.log(lams[1]) - np.log(lams[2]))
    B = np.array(betas) * ys / xs[None, :]
    B[:, ~ju] = 0.0
    a0 = ym - B @ xm
    return GlmnetPath("gaussian", lams * ys, a0, B, np.array(devs), npass_tot)


def _rsq(C, g, a):
    # g = c - C a  (c = X'y), so c = g + C a ; R^2 = 2 a'c - a'C a (ysd'ysd = 1)
    c = g + C @ a
    return float(2 * a @ c - a @ C @ a)


def lognet(X, y, alpha=1.0, penalty_factor=None, lambdas=None, nlambda=100, lambda_min_ratio=None,
           thresh=1e-7, maxit=100000, weights=None):
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64).ravel()
    n, p = X.shape
    w = np.full(n, 1.0 / n) if weights is None else np.asarray(weights, float) / np.sum(weights)
    xm = w @ X
    xs = np.sqrt(np.maximum(w @ (X * X) - xm * xm, 0.0))
    ju = xs > 0
    xs_safe = np.where(ju, xs, 1.0)
    Xs = (X - xm) / xs_safe
    vp = _rescale_pf(penalty_factor, p)
    flmin = lambda_min_ratio if lambda_min_ratio is not None else (1e-4 if n > p else 1e-2)
    q0 = float(w @ y)
    dev0 = _dev(w, y, np.full(n, q0))
    b0 = np.log(q0 / (1 - q0))
    b = np.zeros(p)
    ulam = None if lambdas is None else np.sort(np.asarray(lambdas, float))[::-1]
    nlam = nlambda if ulam is None else len(ulam)
    alf = flmin ** (1.0 / (nlam - 1)) if ulam is None else 1.0
    shr = thresh * dev0
    a0s, betas, lams, devs = [], [], [], []
    alm = 0.0
    npass_tot = 0
    active = np.zeros(p, dtype=bool)

    def working(b0, b):
        eta = b0 + Xs @ b
        q = 1.0 / (1.0 + np.exp(-eta))
        q = np.clip(q, PMIN, 1 - PMIN)
        v = w * q * (1 - q)
        r = w * (y - q)
        return q, v, r

    for m, spec in _lambda_seq_iter(nlam, flmin, ulam):
        if spec is None:
            q, v, r = working(b0, b)
            gfull = Xs.T @ r
            mask = ju & (vp > 0)
            alm = alf * np.max(np.abs(gfull[mask]) / vp[mask]) / max(alpha, 1e-3)
        elif isinstance(spec, str):
            alm *= alf
        else:
            alm = spec
        for _outer in range(1000):
            q, v, r = working(b0, b)
            C = (Xs * v[:, None]).T @ Xs
            xv = np.diag(C).copy()
            cint = Xs.T @ v
            xmz = float(v.sum())
            g = Xs.T @ r
            gint = float(r.sum())
            bs0, bs = b0, b.copy()
            npass, gint, db0, active = cd_solve(C, g, b, vp, xv, alm * alpha, alm * (1 - alpha), shr,
                                                ju, cint=cint, gint=gint, xmz=xmz,
                                                maxit=maxit - npass_tot, state=active)
            npass_tot += npass
            b0 += db0
            dl = max(np.max(xv * (b - bs) ** 2) if p else 0.0, xmz * (b0 - bs0) ** 2)
            if dl < shr:
                break
        q, _, _ = working(b0, b)
        dev = _dev(w, y, q)
        a0s.append(b0)
        betas.append(b.copy())
        lams.append(alm)
        devs.append(1.0 - dev / dev0)
        if ulam is None and m >= MNLAM - 1 and m > 0:
            if devs[-1] - devs[-2] < FDEV * devs[-1] or devs[-1] > DEVMAX:
                break
    lams = np.array(lams)
    if ulam is None and len(lams) >= 3:
        lams[0] = np.exp(2 * np.log(lams[1]) - np.log(lams[2]))
    B = np.array(betas) / xs_safe[None, :]
    B[:, ~ju] = 0.0
    a0 = np.array(a0s) - B @ xm
    return GlmnetPath("binomial", lams, a0, B, np.array(devs), npass_tot)


def _dev(w, y, q):
    q = np.clip(q, PMIN, 1 - PMIN)
    return float(-2.0 * np.sum(w * (y * np.log(q) + (1 - y) * np.log(1 - q))))


def glmnet(X, y, family="gaussian", **kw) -> GlmnetPath:
    if family == "gaussian":
        return elnet_gaussian(X, y, **kw)
    if family == "binomial":
        return lognet(X, y, **kw)
    raise ValueError(family)


@dataclass
class CvGlmnet:
    fit: GlmnetPath
    lambdas: np.ndarray
    cvm: np.ndarray
    cvsd: np.ndarray
    idx_min: int
    idx_1se: int
    foldid: np.ndarray
    fold_fits: list = field(default_factory=list)

    @property
    def lambda_min(self):
        return float(self.lambdas[self.idx_min])

    @property
    def lambda_1se(self):
        return float(self.lambdas[self.idx_1se])

    def index_of(self, s):
        if s in ("lambda.1se", None):
            return self.idx_1se
        if s == "lambda.min":
            return self.idx_min
        s = float(s)
        hit = np.flatnonzero(np.isclose(self.lambdas, s, rtol=1e-12, atol=0))
        if hit.size:
            return int(hit[0])
        raise ValueError("lambda not on path; interpolation not supported")

    def coef(self, s="lambda.1se"):
        """(intercept, beta) — ``coef(cv.glmnet)`` defaults to lambda.1se (Q5)."""
        i = self.index_of(s)
        return float(self.fit.a0[i]), self.fit.beta[i].copy()

    def predict(self, X, s="lambda.1se", type="response"):
        i = self.index_of(s)
        eta = self.fit.predict_link(X, i)
        if type == "response" and self.fit.family == "binomial":
            return 1.0 / (1.0 + np.exp(-eta))
        return eta


def cv_select(lambdas, cvraw, fold_n):
    """cvm / cvsd / lambda.min / lambda.1se from a (K, L) per-fold loss matrix."""
    wts = np.asarray(fold_n, float)
    cvm = (wts[:, None] * cvraw).sum(0) / wts.sum()
    cvsd = np.sqrt((wts[:, None] * (cvraw - cvm) ** 2).sum(0) / wts.sum() / (len(wts) - 1))
    cmin = np.min(cvm)
    idx_min = int(np.flatnonzero(cvm <= cmin)[0])       # lambdas decreasing: first = largest
    idx_1se = int(np.flatnonzero(cvm <= cvm[idx_min] + cvsd[idx_min])[0])
    return cvm, cvsd, idx_min, idx_1se


def fold_loss(family, y, pred):
    if family == "gaussian":
        return (y[:, None] - pred) ** 2
    p = np.clip(pred, PMIN, 1 - PMIN)
    return -2.0 * (y[:, None] * np.log(p) + (1 - y[:, None]) * np.log(1 - p))


def cv_glmnet(X, y, family="gaussian", alpha=1.0, penalty_factor=None, nfolds=10, foldid=None,
              seed=1991, fold_stream=0, keep_fold_fits=False, **kw) -> CvGlmnet:
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64).ravel()
    n = X.shape[0]
    if foldid is None:
        foldid = rng.fold_ids(n, nfolds, seed, fold_stream)
    K = int(foldid.max()) + 1
    full = glmnet(X, y, family=family, alpha=alpha, penalty_factor=penalty_factor, **kw)
    lam = full.lambdas
    cvraw = np.empty((K, len(lam)))
    fold_n = np.empty(K)
    fits = []
    for k in range(K):
        tr = foldid != k
        te = ~tr
        kw2 = {kk: vv for kk, vv in kw.items() if kk not in ("nlambda", "lambda_min_ratio")}
        fk = glmnet(X[tr], y[tr], family=family, alpha=alpha, penalty_factor=penalty_factor,
                    lambdas=lam, **kw2)
        pred = fk.predict(X[te])
        cvraw[k] = fold_loss(family, y[te], pred).mean(0)
        fold_n[k] = te.sum()
        if keep_fold_fits:
            fits.append(fk)
    cvm, cvsd, i_min, i_1se = cv_select(lam, cvraw, fold_n)
    return CvGlmnet(full, lam, cvm, cvsd, i_min, i_1se, foldid, fits)
