"""Float64 reference of approximate residual balancing (E14).

``residual_balance_ATE`` (ate_functions.R:393-405) delegates to
``balanceHD::residualBalance.ate(X, Y, W, estimate.se=TRUE, optimizer=...)``:

* columns scaled by their sample SD (binary columns left alone);
* balance target = column means of the scaled covariates over both arms;
* per arm w: balancing weights
      gamma = argmin (1-zeta)||gamma||^2 + zeta ||M_w' gamma - target||_inf^2
              s.t. sum(gamma) = 1, gamma >= 0            (zeta = 0.5)
  plus ``cv.glmnet(M_w, Y_w, alpha=0.9)`` predicted at lambda.1se;
  mu_w = target . beta_w + sum(gamma * (Y_w - M_w beta_w)),
  var_w = sum(gamma^2 * residual^2);
* tau = mu_1 - mu_0, se = sqrt(var_1 + var_0).

The reference ran the QP through pogs (ADMM, ``ate_replication.Rmd:243``) or
quadprog; both approximate the same optimum. Here it is solved to ~1e-10 by a
Mehrotra predictor-corrector interior-point method whose per-iteration O(n)
work is one weighted Gram of [M 1] (GPU: the K01 kernel) plus a (2p+1)-dim
Cholesky solve — see ``ipm_balance``.
"""
from __future__ import annotations

import numpy as np

from ..parallel import rng
from ..result import AteResult
from . import glmnet as gn


def scale_columns(X):
    """balanceHD ``scale.X``: divide by sd (n-1); binary (0/1) columns keep scale 1."""
    X = np.asarray(X, dtype=np.float64)
    scl = X.std(0, ddof=1)
    binary = np.all((X == 0) | (X == 1), axis=0)
    scl = np.where(binary | (scl == 0), 1.0, scl)
    return X / scl, scl


def _kkt_solve(M, D, W, r_d, r_p, r_g, r_sz, r_gt, s, z, gam, t, allow_negative):
    """Newton step of the balancing QP via the (2p+1) Schur complement.
    Unknown order: x = (gamma[n], delta); inequality rows [M'g - d <= m; -M'g - d <= -m]."""
    n, p = M.shape
    Dg, Dd = D[:n], D[n]
    # rhs1 = -r_d - G'((z r_g - r_sz)/s) - E'(r_gt/gamma)
    v = (z * r_g - r_sz) / s
    rhs1 = -r_d.copy()
    rhs1[:n] -= M @ (v[:p] - v[p:])
    rhs1[n] -= -(v[:p].sum() + v[p:].sum())
    if not allow_negative:
        rhs1[:n] -= r_gt / gam
    # K = B D^-1 B' + diag(1/W, 0), B = [G; A]
    Mw = M / Dg[:, None]
    Smm = M.T @ Mw
    Sm1 = Mw.sum(0)
    S11 = (1.0 / Dg).sum()
    K = np.zeros((2 * p + 1, 2 * p + 1))
    K[:p, :p] = Smm
    K[p:2 * p, p:2 * p] = Smm
    K[:p, p:2 * p] = -Smm
    K[p:2 * p, :p] = -Smm
    K[:p, 2 * p] = Sm1
    K[2 * p, :p] = Sm1
    K[p:2 * p, 2 * p] = -Sm1
    K[2 * p, p:2 * p] = -Sm1
    K[2 * p, 2 * p] = S11
    K[:2 * p, :2 * p] += 1.0 / Dd  # delta column: b_delta = [-1_p; -1_p; 0]
    K[np.arange(2 * p), np.arange(2 * p)] += 1.0 / W
    u = rhs1 / D
    rk = np.empty(2 * p + 1)
    mg = M.T @ u[:n]
    rk[:p] = mg - u[n]
    rk[p:2 * p] = -mg - u[n]
    rk[2 * p] = u[:n].sum() + r_p
    L = np.linalg.cholesky(K)
    sol = np.linalg.solve(L.T, np.linalg.solve(L, rk))
    uu, dy = sol[:2 * p], sol[2 * p]
    # dx = D^-1 (rhs1 - B' [u; dy])
    bt = np.empty(n + 1)
    bt[:n] = M @ (uu[:p] - uu[p:]) + dy
    bt[n] = -(uu.sum())
    dx = (rhs1 - bt) / D
    dz = uu + v
    Gdx = np.concatenate([M.T @ dx[:n] - dx[n], -(M.T @ dx[:n]) - dx[n]])
    ds = -r_g - Gdx
    dt = None if allow_negative else (-r_gt - t * dx[:n]) / gam
    return dx, dy, dz, ds, dt


def _max_step(v, dv):
    neg = dv < 0
    if not np.any(neg):
        return 1.0
    return float(min(1.0, np.min(-v[neg] / dv[neg])))


def ipm_balance(M, target, zeta=0.5, allow_negative=False, tol=1e-11, maxit=100):
    """Balancing weights QP (balanceHD ``approx.balance``) by primal-dual IPM.
    Returns (gamma, info dict)."""
    M = np.asarray(M, dtype=np.float64)
    m = np.asarray(target, dtype=np.float64)
    n, p = M.shape
    Pd = np.r_[np.full(n, 2 * (1 - zeta)), 2 * zeta]
    gam = np.full(n, 1.0 / n)
    delta = np.max(np.abs(M.T @ gam - m)) + 1.0
    x = np.r_[gam, delta]
    y = 0.0
    h = np.r_[m, -m]

    def Gx(x_):
        mg = M.T @ x_[:n]
        return np.r_[mg - x_[n], -mg - x_[n]]

    s = h - Gx(x)
    z = np.ones(2 * p)
    t = np.ones(n) if not allow_negative else None
    it = 0
    for it in range(1, maxit + 1):
        gam = x[:n]
        Gtz = np.empty(n + 1)
        Gtz[:n] = M @ (z[:p] - z[p:])
        Gtz[n] = -z.sum()
        r_d = Pd * x + Gtz
        r_d[:n] += y
        if not allow_negative:
            r_d[:n] -= t
        r_p = gam.sum() - 1.0
        r_g = Gx(x) + s - h
        ncomp = 2 * p + (0 if allow_negative else n)
        mu = (s @ z + (0.0 if allow_negative else gam @ t)) / ncomp
        scale = max(1.0, np.abs(x).max())
        if mu < tol / n and abs(r_p) < tol and np.abs(r_g).max() < tol * scale \
                and np.abs(r_d).max() < tol * scale:
            break
        D = Pd.copy()
        if not allow_negative:
            D[:n] += t / gam
        W = z / s
        # predictor
        r_sz = s * z
        r_gt = None if allow_negative else gam * t
        dx, dy, dz, ds, dt = _kkt_solve(M, D, W, r_d, r_p, r_g, r_sz, r_gt, s, z, gam, t,
                                        allow_negative)
        a = min(_max_step(s, ds), _max_step(z, dz))
        if not allow_negative:
            a = min(a, _max_step(gam, dx[:n]), _max_step(t, dt))
        mu_aff = ((s + a * ds) @ (z + a * dz)
                  + (0.0 if allow_negative else (gam + a * dx[:n]) @ (t + a * dt))) / ncomp
        sigma = (mu_aff / mu) ** 3
        # corrector
        r_sz = s * z + ds * dz - sigma * mu
        if not allow_negative:
            r_gt = gam * t + dx[:n] * dt - sigma * mu
        dx, dy, dz, ds, dt = _kkt_solve(M, D, W, r_d, r_p, r_g, r_sz, r_gt, s, z, gam, t,
                                        allow_negative)
        a = min(_max_step(s, ds), _max_step(z, dz))
        if not allow_negative:
            a = min(a, _max_step(gam, dx[:n]), _max_step(t, dt))
        a = min(1.0, 0.99 * a)
        x = x + a * dx
        y = y + a * dy
        z = z + a * dz
        s = s + a * ds
        if not allow_negative:
            t = t + a * dt
    gam = x[:n]
    obj = (1 - zeta) * gam @ gam + zeta * np.max(np.abs(M.T @ gam - m)) ** 2
    return gam, {"iters": it, "objective": obj, "delta": x[n], "mu": mu}


def balance_objective(M, target, gam, zeta=0.5):
    return (1 - zeta) * gam @ gam + zeta * np.max(np.abs(M.T @ gam - target)) ** 2


def residual_balance_mean(MW, YW, target, zeta=0.5, alpha=0.9, seed=1991, fold_stream=10,
                          nfolds=10, allow_negative=False):
    """balanceHD ``residualBalance.mean``: (mu_hat, var_hat)."""
    gam, info = ipm_balance(MW, target, zeta, allow_negative)
    cv = gn.cv_glmnet(MW, YW, alpha=alpha, nfolds=nfolds, seed=seed, fold_stream=fold_stream)
    a0, beta = cv.coef()  # lambda.1se (Q5)
    mu_lasso = a0 + target @ beta
    resid = YW - (a0 + MW @ beta)
    return mu_lasso + gam @ resid, float(np.sum(gam ** 2 * resid ** 2)), info


def residual_balance_ate(Y, W, X, zeta=0.5, alpha=0.9, seed=1991, fold_streams=(10, 11),
                         scale_x=True, allow_negative=False, method="residual_balancing"):
    """E14 ``residual_balance_ATE`` (ate_functions.R:393-405), estimate.se=TRUE."""
    Y = np.asarray(Y, dtype=np.float64)
    W = np.asarray(W, dtype=np.float64)
    Xs = scale_columns(X)[0] if scale_x else np.asarray(X, dtype=np.float64)
    target = Xs.mean(0)
    t1 = W == 1
    mu1, v1, i1 = residual_balance_mean(Xs[t1], Y[t1], target, zeta, alpha, seed, fold_streams[0],
                                        allow_negative=allow_negative)
    mu0, v0, i0 = residual_balance_mean(Xs[~t1], Y[~t1], target, zeta, alpha, seed,
                                        fold_streams[1], allow_negative=allow_negative)
    return AteResult.make(method, mu1 - mu0, np.sqrt(v1 + v0), mu1=mu1, mu0=mu0,
                          ipm_iters=(i1["iters"], i0["iters"]))
