"""K08/K09 elastic-net ops: glmnet-equivalent gaussian paths + cv.glmnet selection,
computed from per-segment Gram matrices (K01) — no extra pass over the data.

``cv_enet_gaussian`` covers both reference usages:

* plain ``cv.glmnet`` (E5, E6, E11; ``ate_functions.R:101,123,304,305``): one full
  training set = all segments, CV folds = the segments;
* nested cross-fitting (DML nuisances): K full training sets (all segments but
  k), each cross-validated over its own K-1 segments. Training sets that occur
  twice (all \\ {k, s} = all \\ {s, k}) are prepared once.

GPU: ``csrc/enet.hip``. CPU: numpy with the same algorithm (reference core).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from .. import _native
from ..reference import glmnet as ref
from .devconst import const, const_bytes


def _stream():
    return torch.cuda.current_stream().cuda_stream


@dataclass
class EnetCvResult:
    lambdas: torch.Tensor     # [nfull, L] original scale (NaN beyond nlam)
    nlam: torch.Tensor        # [nfull]
    cvm: torch.Tensor         # [nfull, L]
    cvsd: torch.Tensor
    sel: torch.Tensor         # [nfull, 2] (idx_min, idx_1se)
    coef_path: torch.Tensor   # [nfull, L, p+1] original-scale (intercept first)
    coef_min: torch.Tensor    # [nfull, p+1]
    coef_1se: torch.Tensor    # [nfull, p+1]
    full_keys: list           # (full set index, y index) per full problem
    npass: torch.Tensor       # [nfull] passes of the full-data problems
    fold_npass: torch.Tensor | None = None   # [nfold] (< 0: the fold's wait timed out)

    def check(self):
        """Raise NumericalError if any fold path was truncated (host sync). The device
        results are already NaN-poisoned in that case, so graph replays that never call
        this still cannot return a silently different lambda selection."""
        bad = [] if self.fold_npass is None else \
            np.flatnonzero(self.fold_npass.cpu().numpy() < 0).tolist()
        if bad:
            from ..utils.guards import NumericalError
            raise NumericalError(f"CV fold path(s) {bad} timed out waiting for their "
                                 "full-data lambda sequence; selection is invalid")
        return self


def poison_if_truncated(fold_npass: torch.Tensor, *ts):
    """NaN every tensor in ``ts`` when any fold path of the launch was truncated
    (device-side, capturable: no host sync)."""
    bad = (fold_npass < 0).any()
    nan = torch.full((), float("nan"), dtype=torch.float64, device=fold_npass.device)
    return [torch.where(bad, nan, t) for t in ts]


def _zeroed(dev, *specs):
    """Zero-filled tensors (shape, dtype) carved from ONE buffer: one fill launch instead of
    one per tensor (they sit on the single call's critical path; 256-B aligned views)."""
    sizes = [int(np.prod(sh)) * torch.empty((), dtype=dt).element_size() for sh, dt in specs]
    offs = np.concatenate([[0], np.cumsum([(b + 255) // 256 * 256 for b in sizes])])
    buf = torch.zeros(int(offs[-1]), dtype=torch.uint8, device=dev)
    return [buf[int(o):int(o) + b].view(dt).view(sh)
            for (sh, dt), o, b in zip(specs, offs[:-1], sizes)]


def _rescale_vp(vp, p):
    vp = np.ones(p) if vp is None else np.maximum(np.asarray(vp, float), 0)
    return vp * p / vp.sum()


def cv_enet_gaussian(G: torch.Tensor, panel, xcols, ycols, full_sets=None, penalty_factor=None,
                     alpha=1.0, nlambda=100, lambda_min_ratio=None, thresh=1e-7,
                     maxit=100000, seg_counts=None) -> EnetCvResult:
    """Cross-validated gaussian elastic net from the segment Gram stack ``G`` [nseg,P,P].

    full_sets: list of lists of segment ids (default: one set with all segments).
    seg_counts: rows per segment (default: the panel's; pass the GLOBAL counts when G
    was all-reduced over row shards). Problems are ordered (full set f, y index)."""
    nseg = G.shape[0]
    P = G.shape[1]
    p = len(xcols)
    ny = len(ycols)
    if full_sets is None:
        full_sets = [list(range(nseg))]
    # training sets: each full set, then every (full set minus one segment)
    tsets, tindex = [], {}

    def tid(segs):
        key = tuple(sorted(segs))
        if key not in tindex:
            tindex[key] = len(tsets)
            tsets.append(key)
        return tindex[key]

    full_t = [tid(fs) for fs in full_sets]
    fold_t, fold_hold = [], []
    for fs in full_sets:
        for s in fs:
            fold_t.append(tid([q for q in fs if q != s]))
            fold_hold.append(s)
    K = len(full_sets[0])
    assert all(len(fs) == K for fs in full_sets), "full sets must have equal fold counts"
    masks = np.zeros((len(tsets), nseg), dtype=np.uint8)
    for i, ts in enumerate(tsets):
        masks[i, list(ts)] = 1
    nreal = np.asarray(panel.seg_nreal if seg_counts is None else seg_counts, dtype=np.float64)
    n_full = [nreal[list(fs)].sum() for fs in full_sets]
    if lambda_min_ratio is None:
        lambda_min_ratio = 1e-4 if min(n_full) > p else 1e-2
    vp = _rescale_vp(penalty_factor, p)
    L = nlambda
    # problem tables
    full_probs = [(full_t[f], y, -1, nlambda) for f in range(len(full_sets)) for y in range(ny)]
    full_keys = [(f, y) for f in range(len(full_sets)) for y in range(ny)]
    fold_probs, fold_ycol, fold_holds, fold_of_full = [], [], [], []
    for f in range(len(full_sets)):
        for k in range(K):
            for y in range(ny):
                src = f * ny + y
                fold_probs.append((fold_t[f * K + k], y, src, 0))
                fold_ycol.append(ycols[y])
                fold_holds.append(fold_hold[f * K + k])
    # fold_probs index for (full problem fp, k): order above is f, k, y
    fold_index = np.zeros((len(full_probs), K), dtype=np.int32)
    nfold = np.zeros((len(full_probs), K))
    for f in range(len(full_sets)):
        for k in range(K):
            for y in range(ny):
                fold_index[f * ny + y, k] = (f * K + k) * ny + y
                nfold[f * ny + y, k] = nreal[fold_hold[f * K + k]]
    # group fold problems by training set (the path kernel places consecutive problems
    # on the same XCD, so problems sharing a Gram share an L2)
    perm = np.argsort([fp[0] for fp in fold_probs], kind="stable")
    inv = np.empty_like(perm)
    inv[perm] = np.arange(len(perm))
    fold_probs = [fold_probs[i] for i in perm]
    fold_ycol = [fold_ycol[i] for i in perm]
    fold_holds = [fold_holds[i] for i in perm]
    fold_index = inv[fold_index].astype(np.int32)
    if G.is_cuda:
        return _cv_gpu(G, P, nseg, masks, xcols, ycols, p, ny, vp, panel.cols["one"], full_probs,
                       fold_probs, fold_ycol, fold_holds, fold_index, nfold, alpha,
                       lambda_min_ratio, thresh, maxit, L, full_keys, panel.dtype)
    return _cv_cpu(G, masks, xcols, ycols, p, ny, vp, panel.cols["one"], full_probs, fold_probs,
                   fold_ycol, fold_holds, fold_index, nfold, alpha, lambda_min_ratio, thresh, maxit,
                   L, full_keys)


_PROB_DT = np.dtype([("train", "<i4"), ("y", "<i4"), ("src", "<i4"), ("nlam", "<i4")])


def _probs_tensor(probs, dev):
    return const_bytes(np.array(probs, dtype=_PROB_DT), dev)


def _cv_gpu(G, P, nseg, masks, xcols, ycols, p, ny, vp, one, full_probs, fold_probs, fold_ycol,
            fold_holds, fold_index, nfold, alpha, flmin, thresh, maxit, L, full_keys,
            panel_dtype):
    dev = G.device
    s = _stream()
    f64 = dict(dtype=torch.float64, device=dev)
    nt = masks.shape[0]
    masks_t = const(masks, torch.uint8, dev)
    xc = const(xcols, torch.int32, dev)
    yc = const(ycols, torch.int32, dev)
    c_f32 = int(panel_dtype != torch.float64)
    ldc = (p + 63) // 64 * 64   # zero-padded row stride (16-B aligned row segments)
    nf = len(full_probs)
    probs_all = list(full_probs) + list(fold_probs)
    nq = len(probs_all)
    i32 = torch.int32
    C, apath, rsq, nlam, npass, progress = _zeroed(
        dev, ((nt, p, ldc), torch.float32 if c_f32 else torch.float64), ((nq, L, p), torch.float64),
        ((nq, L), torch.float64), ((nq,), i32), ((nq,), i32), ((nq,), i32))
    g = torch.empty((nt, ny, p), **f64)
    xm = torch.empty((nt, p), **f64)
    xs = torch.empty((nt, p), **f64)
    ju = torch.empty((nt, p), dtype=torch.uint8, device=dev)
    ym = torch.empty((nt, ny), **f64)
    ys = torch.empty((nt, ny), **f64)
    nobs = torch.empty(nt, **f64)
    _native.call("ate_enet_prepare", G.data_ptr(), nseg, P, masks_t.data_ptr(), nt, xc.data_ptr(),
                 p, one, yc.data_ptr(), ny, C.data_ptr(), c_f32, g.data_ptr(), xm.data_ptr(),
                 xs.data_ptr(), ju.data_ptr(), ym.data_ptr(), ys.data_ptr(), nobs.data_ptr(), s)
    vp_t = const(np.asarray(vp, dtype=np.float64), torch.float64, dev)
    # ONE launch: full problems [0, nf) + fold problems [nf, nq); fold problems consume
    # their source's lambda sequence as it is published (device-side progress flags)
    pr = _probs_tensor(probs_all, dev)
    lams = torch.full((nq, L), float("nan"), **f64)
    # each full problem's whole lambda sequence, published at its lambda 1 for the folds
    lampub = torch.empty((nq, L), **f64)
    _native.call("ate_enet_path", C.data_ptr(), c_f32, g.data_ptr(), p, ny, ju.data_ptr(),
                 ys.data_ptr(), vp_t.data_ptr(), pr.data_ptr(), nq, alpha, flmin, thresh,
                 maxit, apath.data_ptr(), lams.data_ptr(), rsq.data_ptr(), nlam.data_ptr(),
                 npass.data_ptr(), L, progress.data_ptr(), lampub.data_ptr(), s)
    coef = torch.empty((nq, L, p + 1), **f64)
    _native.call("ate_enet_coef", apath.data_ptr(), pr.data_ptr(), nq, p, ny, L,
                 nlam.data_ptr(), xm.data_ptr(), xs.data_ptr(), ju.data_ptr(), ym.data_ptr(),
                 ys.data_ptr(), coef.data_ptr(), s)
    hold = const([0] * nf + list(fold_holds), torch.int32, dev)
    ycol_p = const([0] * nf + list(fold_ycol), torch.int32, dev)
    cvraw = torch.empty((nq, L), **f64)
    _native.call("ate_enet_cvloss_gauss", G.data_ptr(), P, hold.data_ptr(), xc.data_ptr(), p, one,
                 ycol_p.data_ptr(), coef.data_ptr(), nlam.data_ptr(), L, nf, nq - nf,
                 cvraw.data_ptr(), s)
    fidx = const(fold_index + nf, torch.int32, dev)
    nfold_t = const(nfold, torch.float64, dev)
    cvm = torch.empty((nf, L), **f64)
    cvsd = torch.empty((nf, L), **f64)
    sel = torch.empty((nf, 2), dtype=torch.int32, device=dev)
    K = fold_index.shape[1]
    # a fold whose spin on its source's progress flag timed out (npass = -1; csrc/enet.hip)
    # has a truncated path: cvm, and so lambda.min / lambda.1se, would silently change --
    # the select and pick kernels NaN-poison cvm / cvsd / the picked coefficients then
    fold_npass = npass[nf:]
    _native.call("ate_cv_select", cvraw.data_ptr(), fidx.data_ptr(), nfold_t.data_ptr(), K, nf,
                 nlam.data_ptr(), L, cvm.data_ptr(), cvsd.data_ptr(), sel.data_ptr(),
                 fold_npass.data_ptr(), nq - nf, s)
    cmin = torch.empty((nf, p + 1), **f64)
    c1se = torch.empty((nf, p + 1), **f64)
    _native.call("ate_enet_pick", coef.data_ptr(), sel.data_ptr(), p, L, nf, cmin.data_ptr(),
                 c1se.data_ptr(), fold_npass.data_ptr(), nq - nf, s)
    return EnetCvResult(lams[:nf], nlam[:nf], cvm, cvsd, sel, coef[:nf], cmin, c1se, full_keys,
                        npass[:nf], fold_npass)


def _cv_cpu(G, masks, xcols, ycols, p, ny, vp, one, full_probs, fold_probs, fold_ycol, fold_holds,
            fold_index, nfold, alpha, flmin, thresh, maxit, L, full_keys):
    Gn = G.double().cpu().numpy()
    nt = masks.shape[0]
    stats = []
    for t in range(nt):
        Gt = np.tensordot(masks[t].astype(float), Gn, axes=1)
        n = Gt[one, one]
        sx = Gt[one, xcols] / n
        vx = np.diag(Gt)[xcols] / n - sx * sx
        ju = vx > 0
        xs = np.where(ju, np.sqrt(np.maximum(vx, 0)), 1.0)
        Cm = (Gt[np.ix_(xcols, xcols)] / n - np.outer(sx, sx)) / np.outer(xs, xs)
        Cm[~ju, :] = 0
        Cm[:, ~ju] = 0
        Cm[np.flatnonzero(~ju), np.flatnonzero(~ju)] = 1.0
        gs, ymv, ysv = [], [], []
        for yc in ycols:
            my = Gt[one, yc] / n
            vy = Gt[yc, yc] / n - my * my
            sy = np.sqrt(vy) if vy > 0 else 1.0
            gj = np.where(ju, (Gt[xcols, yc] / n - sx * my) / (xs * sy), 0.0)
            gs.append(gj)
            ymv.append(my)
            ysv.append(sy)
        stats.append(dict(C=Cm, g=gs, xm=sx, xs=xs, ju=ju, ym=ymv, ys=ysv, n=n))

    def run(probs, src_paths):
        res = []
        for (t, y, src, nlam_req) in probs:
            st = stats[t]
            lam = None if src < 0 else src_paths[src].lambdas
            path = ref._elnet_core(st["C"], st["g"][y], np.ones(p), st["xm"], st["xs"], st["ym"][y],
                                   st["ys"][y], st["ju"], alpha, vp, lam, nlam_req or L, flmin,
                                   thresh, maxit)
            res.append(path)
        return res

    full = run(full_probs, None)
    folds = run(fold_probs, full)
    nf = len(full_probs)
    K = fold_index.shape[1]
    lams = np.full((nf, L), np.nan)
    nlam = np.zeros(nf, dtype=np.int32)
    coef = np.full((nf, L, p + 1), np.nan)
    for f, path in enumerate(full):
        m = len(path.lambdas)
        lams[f, :m] = path.lambdas
        nlam[f] = m
        coef[f, :m, 0] = path.a0
        coef[f, :m, 1:] = path.beta
    cvraw = np.full((len(fold_probs), L), np.nan)
    for q, path in enumerate(folds):
        Gh = Gn[fold_holds[q]]
        yc = fold_ycol[q]
        n = Gh[one, one]
        for m in range(len(path.lambdas)):
            a0, b = path.a0[m], path.beta[m]
            Gxx = Gh[np.ix_(xcols, xcols)]
            sse = (Gh[yc, yc] - 2 * a0 * Gh[one, yc] - 2 * b @ Gh[xcols, yc] + n * a0 * a0
                   + 2 * a0 * b @ Gh[xcols, one] + b @ Gxx @ b)
            cvraw[q, m] = sse / n
    cvm = np.full((nf, L), np.nan)
    cvsd = np.full((nf, L), np.nan)
    sel = np.zeros((nf, 2), dtype=np.int32)
    for f in range(nf):
        m = nlam[f]
        raw = cvraw[fold_index[f]][:, :m]
        cm, cs, i0, i1 = ref.cv_select(lams[f, :m], raw, nfold[f])
        cvm[f, :m], cvsd[f, :m] = cm, cs
        sel[f] = (i0, i1)
    cmin = np.stack([coef[f, sel[f, 0]] for f in range(nf)])
    c1se = np.stack([coef[f, sel[f, 1]] for f in range(nf)])
    t = torch.from_numpy
    return EnetCvResult(t(lams), t(nlam), t(cvm), t(cvsd), t(sel), t(coef), t(cmin), t(c1se),
                        full_keys, t(np.array([pth.npasses for pth in full])))
