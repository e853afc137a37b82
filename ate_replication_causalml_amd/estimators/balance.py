"""Device approximate residual balancing (E14; ate_functions.R:393-405 ->
balanceHD::residualBalance.ate).

Both arms share ONE fold-segmented panel (segments 0..K-1 = treated folds,
K..2K-1 = control folds), so

* the per-arm ``cv.glmnet(alpha=0.9)`` fits are two "full sets" of a single
  ``cv_enet_gaussian`` call on one Gram stack (K01 + K08/K09);
* the balancing QPs of both arms run in lock-step through one interior-point
  loop whose O(n) work per iteration is ONE weighted Gram launch over the whole
  panel (segment-summed per arm) plus two GEMVs; the (2p+1)-dim Schur systems
  are batched over the arms.

Matches reference/balance.py (same algorithm, both solved to ~1e-10).
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import gemv
from ..ops.devconst import const
from ..ops.enet import cv_enet_gaussian
from ..ops.gram import gram
from ..ops.linalg import spd_solve
from ..ops.panel import build_panel
from ..parallel import rng
from ..reference.balance import scale_columns
from ..result import AteResult
from ..utils.graphs import estimator_graphs
from .common import as_np, resolve_device


def _arm_masks(pan, K):
    valid = pan.valid() != 0
    m = torch.zeros(2, pan.ld, dtype=torch.bool, device=pan.device)
    for a in range(2):
        for s in range(a * K, (a + 1) * K):
            r0, r1 = pan.seg_bounds[s]
            m[a, r0:r1] = valid[r0:r1]
    return m


def _schur(Garm, xc, one, Dd, W, p):
    """Batched K = B D^-1 B' + diag(1/W, 0) from the per-arm weighted Gram [2,P,P]."""
    Smm = Garm[:, xc][:, :, xc]
    Sm1 = Garm[:, xc, one]
    S11 = Garm[:, one, one]
    A = Garm.shape[0]
    K = torch.zeros(A, 2 * p + 1, 2 * p + 1, dtype=Garm.dtype, device=Garm.device)
    K[:, :p, :p] = Smm
    K[:, p:2 * p, p:2 * p] = Smm
    K[:, :p, p:2 * p] = -Smm
    K[:, p:2 * p, :p] = -Smm
    K[:, :p, 2 * p] = Sm1
    K[:, 2 * p, :p] = Sm1
    K[:, p:2 * p, 2 * p] = -Sm1
    K[:, 2 * p, p:2 * p] = -Sm1
    K[:, 2 * p, 2 * p] = S11
    K[:, :2 * p, :2 * p] += (1.0 / Dd)[:, None, None]
    # diagonal view, not K[:, range, range]: a host index tensor is not capturable
    torch.diagonal(K, dim1=1, dim2=2)[:, :2 * p] += 1.0 / W
    return K


def ipm_balance_panel(pan, masks, target, zeta=0.5, tol=1e-11, maxit=100, seg_arm=None,
                      fixed=False, allow_negative=False):
    """Balancing weights for every arm a (rows ``masks[a]``) toward ``target`` [p].
    Returns gamma [ld] (each row carries its own arm's weight) and iteration counts.

    ``fixed``: no host sync at all (hipGraph capture): run all ``maxit`` iterations; an
    arm's state is frozen (``torch.where``, so a NaN from a degenerate post-convergence
    Newton system cannot leak into it) from the iteration at which it converged, and the
    iteration counts come back as a device tensor. ``seg_arm`` (host, per segment: arm or
    -1) then has to be given, since deriving it from ``masks`` reads the device.

    ``allow_negative``: drop gamma >= 0 (balanceHD ``allow.negative.weights``): no row
    barrier (t), the step length is limited by the (s, z) pairs only
    (reference/balance.ipm_balance, same algorithm)."""
    neg = bool(allow_negative)
    dev, dt = pan.device, torch.float64
    xc = const(pan.xcols, torch.int64, dev)
    one = pan.cols["one"]
    p = len(pan.xcols)
    A = masks.shape[0]
    mf = masks.to(dt)                                   # [A, ld]
    live = masks.any(0)
    lf = live.to(dt)
    nA = mf.sum(1)
    m = target.to(dev, dt)
    h = torch.cat([m, -m])
    if seg_arm is None:
        seg_arm = torch.full((pan.nseg,), -1, dtype=torch.long)
        for a in range(A):
            for s in range(pan.nseg):
                r0, r1 = pan.seg_bounds[s]
                if r1 > r0 and bool(masks[a, r0:r1].any()):
                    seg_arm[s] = a
    seg_arm = torch.as_tensor(seg_arm, dtype=torch.long)
    arm_of = [const((seg_arm == a).tolist(), torch.bool, dev) for a in range(A)]

    grp = torch.full((pan.ld,), -1, dtype=torch.int8, device=dev)
    for a in range(A):
        grp = torch.where(masks[a], torch.full_like(grp, a), grp)

    def per_arm_T(v):            # M_a' v over each arm's rows -> [A, p]
        return gemv.xtv(pan, pan.xcols, v, grp, A)

    def rows_from(V):            # row i of arm a: M_i . V[a] -> [ld]
        return gemv.xv(pan, pan.xcols, V, grp)

    def arm_sum(v):
        return (mf * v).sum(1)

    def Gx(gam, delta):
        mg = per_arm_T(gam)
        return torch.cat([mg - delta[:, None], -mg - delta[:, None]], 1)

    c_g, c_d = 2 * (1 - zeta), 2 * zeta
    gam = lf * (mf / nA[:, None]).sum(0) + (1 - lf)    # padding rows: 1 (masked everywhere)
    delta = (per_arm_T(gam) - m).abs().amax(1) + 1.0
    y = torch.zeros(A, dtype=dt, device=dev)
    s = h[None] - Gx(gam, delta)
    z = torch.ones(A, 2 * p, dtype=dt, device=dev)
    t = torch.ones(pan.ld, dtype=dt, device=dev)
    ncomp = 2 * p + (0 * nA if neg else nA)
    done = torch.zeros(A, dtype=torch.bool, device=dev)
    iters = np.zeros(A, dtype=int)
    iters_dev = torch.zeros(A, dtype=torch.int64, device=dev)

    def solve(Dg, Dd, W, r_d_g, r_d_d, r_p, r_g, r_sz, r_gt):
        v = (z * r_g - r_sz) / s                                   # [A, 2p]
        rhs_g = lf * (-r_d_g - rows_from(v[:, :p] - v[:, p:]) - (0.0 if neg else r_gt / gam))
        rhs_d = -r_d_d + v.sum(1)
        wts = lf / Dg
        Gs = gram(pan, w=wts.to(pan.data.dtype))                  # [nseg, P, P]
        # per-arm sum of the segment Grams as a fixed-order reduction (index_add_ on a GPU
        # adds with atomics: run-to-run rounding noise the interior point amplifies)
        Garm = torch.stack([torch.where(arm_of[a][:, None, None], Gs, torch.zeros_like(Gs)).sum(0)
                            for a in range(A)])
        K = _schur(Garm, xc, one, Dd, W, p)
        u_g = rhs_g / Dg
        u_d = rhs_d / Dd
        mg = per_arm_T(u_g)
        rk = torch.cat([mg - u_d[:, None], -mg - u_d[:, None], (arm_sum(u_g) + r_p)[:, None]], 1)
        sol = spd_solve(K, rk)
        # a converged arm's Schur system may have lost its positive pivots (spd_solve then
        # returns NaN); its step is discarded anyway, but dy enters every row through the
        # mask product below (0 * NaN = NaN), so zero it before use
        sol = torch.where(done[:, None], torch.zeros_like(sol), sol)
        uu, dy = sol[:, :2 * p], sol[:, 2 * p]
        dxg = lf * (rhs_g - rows_from(uu[:, :p] - uu[:, p:]) - (mf * dy[:, None]).sum(0)) / Dg
        dxd = (rhs_d + uu.sum(1)) / Dd
        dz = uu + v
        mdx = per_arm_T(dxg)
        ds = -r_g - torch.cat([mdx - dxd[:, None], -mdx - dxd[:, None]], 1)
        dtt = torch.zeros_like(gam) if neg else lf * (-r_gt - t * dxg) / gam
        return dxg, dxd, dy, dz, ds, dtt

    def step(vr, dv, vs, dvs):
        """Per-arm max step keeping row vectors (masked) and arm vectors positive."""
        inf = torch.full_like(vr, float("inf"))
        rr = torch.where(dv < 0, -vr / dv, inf)
        ra = torch.stack([torch.where(masks[a], rr, inf).amin() for a in range(A)])
        rs = torch.where(dvs < 0, -vs / dvs, torch.full_like(vs, float("inf"))).amin(1)
        return torch.minimum(torch.minimum(ra, rs), torch.ones_like(ra))

    def step_sz(vs, dvs):
        rs = torch.where(dvs < 0, -vs / dvs, torch.full_like(vs, float("inf"))).amin(1)
        return torch.minimum(rs, torch.ones_like(rs))

    def max_step(ds, dz, dxg, dtt):
        if neg:
            return step_sz(torch.cat([s, z], 1), torch.cat([ds, dz], 1))
        return torch.minimum(step(gam, dxg, torch.cat([s, z], 1), torch.cat([ds, dz], 1)),
                             step(t, dtt, s, ds))

    for it in range(1, maxit + 1):
        r_d_g = lf * (c_g * gam + rows_from(z[:, :p] - z[:, p:]) + (mf * y[:, None]).sum(0)
                      - (0.0 if neg else t))
        r_d_d = c_d * delta - z.sum(1)
        r_p = arm_sum(gam) - 1.0
        r_g = Gx(gam, delta) + s - h[None]
        mu = ((s * z).sum(1) + (0.0 if neg else arm_sum(gam * t))) / ncomp
        scale = torch.clamp(torch.maximum(arm_sum(gam.abs()) * 0 + delta.abs(),
                                          torch.ones_like(delta)), min=1.0)
        rdmax = torch.stack([torch.where(masks[a], r_d_g.abs(), torch.zeros_like(r_d_g)).amax()
                             for a in range(A)])
        conv = (mu < tol / nA) & (r_p.abs() < tol) & (r_g.abs().amax(1) < tol * scale) \
            & (rdmax < tol * scale) & (r_d_d.abs() < tol * scale)
        if fixed:
            done = done | conv
            iters_dev = iters_dev + (~done).long()
        else:
            done_h = (done | conv).cpu().numpy()
            iters[~done_h] = it
            done = done | conv
            if bool(done_h.all()):
                break
        Dg = c_g + (0.0 * gam if neg else t / gam)
        Dd = torch.full((A,), c_d, dtype=dt, device=dev)
        W = z / s
        dxg, dxd, dy, dz, ds, dtt = solve(Dg, Dd, W, r_d_g, r_d_d, r_p, r_g, s * z, lf * gam * t)
        a_aff = max_step(ds, dz, dxg, dtt)
        af = (mf * a_aff[:, None]).sum(0)
        mu_aff = (((s + a_aff[:, None] * ds) * (z + a_aff[:, None] * dz)).sum(1)
                  + (0.0 if neg else arm_sum((gam + af * dxg) * (t + af * dtt)))) / ncomp
        sigma = (mu_aff / mu) ** 3
        sm = (mf * (sigma * mu)[:, None]).sum(0)
        r_sz = s * z + ds * dz - (sigma * mu)[:, None]
        r_gt = lf * (gam * t + dxg * dtt - sm)
        dxg, dxd, dy, dz, ds, dtt = solve(Dg, Dd, W, r_d_g, r_d_d, r_p, r_g, r_sz, r_gt)
        a = max_step(ds, dz, dxg, dtt)
        a = torch.where(done, torch.zeros_like(a), torch.clamp(0.99 * a, max=1.0))
        af = (mf * a[:, None]).sum(0)
        if fixed:
            # freeze converged arms with where (0 * NaN would not be 0)
            frow = (mf * done.to(dt)[:, None]).sum(0) > 0
            gam = torch.where(frow, gam, gam + af * dxg)
            t = torch.where(frow, t, t + af * dtt)
            delta = torch.where(done, delta, delta + a * dxd)
            y = torch.where(done, y, y + a * dy)
            z = torch.where(done[:, None], z, z + a[:, None] * dz)
            s = torch.where(done[:, None], s, s + a[:, None] * ds)
            continue
        gam = gam + af * dxg
        t = t + af * dtt
        delta = delta + a * dxd
        y = y + a * dy
        z = z + a[:, None] * dz
        s = s + a[:, None] * ds
    if fixed:
        return gam * lf, iters_dev
    return gam * lf, iters


class _Budget:
    """Interior-point iteration budget of one panel layout's captured graph (identity-
    hashed: the same object is the GraphCache static argument on every call)."""

    def __init__(self):
        self.value = None


_budgets: dict = {}


def _arb_body(pan, target, zeta, alpha, K, seg_arm, allow_negative=False, budget=None):
    """E14 as one device function (utils/graphs.GraphCache): per-arm CV elastic net, the
    balancing QPs and the residual-balancing estimate. Returns [mu1, mu0, var1, var0,
    iters1, iters0, min fold passes].

    The interior point of a captured graph runs a FIXED budget of iterations (converged
    arms frozen on the device: the same result as stopping). The budget is learned: the
    first call of a layout (eager, the GraphCache warm-up) stops at convergence and sets
    ``budget.value`` to its iteration count plus a margin, so a replay costs about the
    converged iterations, not the 100-iteration worst case."""
    G = gram(pan).clone()
    cv = cv_enet_gaussian(G, pan, pan.xcols, [pan.cols["Y"]],
                          full_sets=[list(range(K)), list(range(K, 2 * K))], alpha=alpha)
    masks = _arm_masks(pan, K)
    tg = target.to(pan.device, torch.float64)
    if budget is not None and budget.value is None and not torch.cuda.is_current_stream_capturing():
        gam, it_h = ipm_balance_panel(pan, masks, tg, zeta, seg_arm=seg_arm,
                                      allow_negative=allow_negative)
        budget.value = int(max(it_h)) + max(4, int(max(it_h)) // 2)
        iters = torch.as_tensor(np.asarray(it_h, dtype=np.int64), device=pan.device)
    else:
        maxit = budget.value if budget is not None and budget.value else 100
        gam, iters = ipm_balance_panel(pan, masks, tg, zeta, seg_arm=seg_arm, fixed=True,
                                       maxit=maxit, allow_negative=allow_negative)
    b = cv.coef_1se.to(torch.float64)
    Xd = pan.data.double()
    fit = b[:, :1] + b[:, 1:] @ Xd.index_select(0, const(pan.xcols, torch.int64, pan.device))
    resid = Xd[pan.cols["Y"]][None] - fit
    mf = masks.double()
    mu = b[:, 0] + b[:, 1:] @ tg + (mf * gam * resid).sum(1)
    var = (mf * gam ** 2 * resid ** 2).sum(1)
    fnp = cv.fold_npass.min().double().reshape(1) if cv.fold_npass is not None else \
        torch.zeros(1, dtype=torch.float64, device=pan.device)
    return torch.cat([mu, var, iters.double(), fnp])


def residual_balance(Y, W, X, zeta=0.5, alpha=0.9, seed=1991, fold_streams=(10, 11), nfolds=10,
                     scale_x=True, method="residual_balancing", device=None, dtype="f64",
                     graph=True, allow_negative=False):
    """E14 on the device; matches reference.balance.residual_balance_ate.

    graph=True (default, GPU): one hipGraph launch per call after the first of a panel
    layout (utils/graphs.GraphCache over _arb_body). The captured interior point runs the
    budget learned by the layout's first call (its converged iteration count plus a
    margin), converged arms frozen on the device, so it equals the stopping solver; a
    replay whose arms did not converge within the budget is redone eagerly and the budget
    raised (the next call recaptures)."""
    dev = resolve_device(device)
    Yn, Wn = as_np(Y), as_np(W)
    Xs = scale_columns(as_np(X))[0] if scale_x else as_np(X)
    target = torch.as_tensor(Xs.mean(0))
    arm = (Wn == 1)
    seg = np.empty(len(Yn), dtype=np.int64)
    seg[arm] = rng.fold_ids(int(arm.sum()), nfolds, seed, fold_streams[0])
    seg[~arm] = nfolds + rng.fold_ids(int((~arm).sum()), nfolds, seed, fold_streams[1])
    pan = build_panel(Xs, None, Yn, folds=seg, dtype=dtype, device=dev)
    if graph and pan.data.is_cuda:
        from ..utils.graphs import layout_key
        K = nfolds
        nr = np.asarray(pan.seg_nreal)
        seg_arm = tuple(int(s // K) if nr[s] > 0 else -1 for s in range(pan.nseg))
        statics = (float(zeta), float(alpha), K, seg_arm, bool(allow_negative))
        bkey = (layout_key(pan), statics)
        budget = _budgets.setdefault(bkey, _Budget())
        out, g = estimator_graphs.run("arb", _arb_body, (pan, target.to(dev)), *statics, budget)
        v = out.cpu().numpy()
        if v[6] < 0:
            from ..utils.guards import NumericalError
            raise NumericalError("CV fold path timed out waiting for its full-data lambda "
                                 "sequence; selection is invalid")
        if budget.value is not None and max(v[4], v[5]) >= budget.value:
            # an arm did not converge within the captured budget: redo this call with the
            # stopping solver and recapture next time with a larger budget
            estimator_graphs.drop("arb", (pan, target.to(dev)), *statics, budget)
            budget.value = None
            return residual_balance(Y, W, X, zeta, alpha, seed, fold_streams, nfolds, scale_x,
                                    method, device, dtype, graph=False,
                                    allow_negative=allow_negative)
        return AteResult.make(method, v[0] - v[1], float(np.sqrt(v[2] + v[3])), mu1=float(v[0]),
                              mu0=float(v[1]), ipm_iters=(int(v[4]), int(v[5])), hipgraph=g,
                              ipm_budget=budget.value)
    G = gram(pan).clone()
    K = nfolds
    cv = cv_enet_gaussian(G, pan, pan.xcols, [pan.cols["Y"]],
                          full_sets=[list(range(K)), list(range(K, 2 * K))], alpha=alpha).check()
    masks = _arm_masks(pan, K)
    gam, iters = ipm_balance_panel(pan, masks, target, zeta, allow_negative=allow_negative)
    b = cv.coef_1se.to(torch.float64)                      # [2, p+1]: arm 1, arm 0
    Xd = pan.data.double()
    fit = b[:, :1] + b[:, 1:] @ Xd[pan.xcols]              # [2, ld]
    resid = Xd[pan.cols["Y"]][None] - fit
    mf = masks.double()
    mu = b[:, 0] + b[:, 1:] @ target.to(dev, torch.float64) + (mf * gam * resid).sum(1)
    var = (mf * gam ** 2 * resid ** 2).sum(1)
    mu, var = mu.cpu().numpy(), var.cpu().numpy()
    return AteResult.make(method, mu[0] - mu[1], float(np.sqrt(var.sum())), mu1=float(mu[0]),
                          mu0=float(mu[1]), ipm_iters=tuple(int(i) for i in iters))
