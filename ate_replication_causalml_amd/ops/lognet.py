"""Binomial elastic net + cv.glmnet on the device (csrc/lognet.hip).

``cv_lognet`` fits the full problem (all segments) and the K fold problems (all
segments but k, on the full problem's lambda sequence), evaluates held-out binomial
deviance per (fold, lambda), and applies the cv.glmnet selection rules
(``ate_cv_select``, shared with the gaussian path). Three launches + selection, no
host synchronisation. CPU tensors run reference/glmnet.py on the same folds.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from .. import _native
from ..reference import glmnet as ref
from .panel import dtype_code


@dataclass
class LognetCvResult:
    lambdas: torch.Tensor    # [L] (NaN beyond nlam)
    nlam: torch.Tensor       # [1] int32
    cvm: torch.Tensor        # [L]
    cvsd: torch.Tensor
    sel: torch.Tensor        # [2] (idx_min, idx_1se)
    coef_path: torch.Tensor  # [L, p+1] original scale, intercept first
    coef_min: torch.Tensor   # [p+1]
    coef_1se: torch.Tensor
    npass: torch.Tensor      # [1 + K]: full fit, then the K fold fits (< 0: wait timed out)

    def check(self):
        """Raise NumericalError if a fold fit was truncated (its wait for the full fit's
        lambda timed out). Device outputs are NaN-poisoned in that case already."""
        bad = np.flatnonzero(self.npass.cpu().numpy()[1:] < 0).tolist()
        if bad:
            from ..utils.guards import NumericalError
            raise NumericalError(f"binomial CV fold fit(s) {bad} timed out waiting for the "
                                 "full fit's lambda sequence; selection is invalid")
        return self


def _rescale_vp(vp, p):
    vp = np.ones(p) if vp is None else np.maximum(np.asarray(vp, float), 0)
    return vp * p / vp.sum()


def cv_lognet(panel, xcols, ycol, penalty_factor=None, alpha=1.0, nlambda=100,
              lambda_min_ratio=None, thresh=1e-7, maxit=100000,
              concurrent=True) -> LognetCvResult:
    """cv.glmnet(x, y, family="binomial") with the panel's segments as the CV folds.

    ``concurrent``: full and fold fits in one launch (fold paths follow the full fit's
    lambdas through device flags); False = two launches, full fit then folds. Same bits.
    ``npass`` < 0 flags a fold whose wait for the full fit timed out."""
    K = panel.nseg
    p = len(xcols)
    n = int(np.sum(panel.seg_nreal))
    flmin = lambda_min_ratio if lambda_min_ratio is not None else (1e-4 if n > p else 1e-2)
    vp = _rescale_vp(penalty_factor, p)
    if not panel.data.is_cuda:
        return _cv_cpu(panel, xcols, ycol, vp, alpha, nlambda, flmin, thresh, maxit)
    if p > 96:
        raise ValueError("device lognet supports p <= 96")
    if panel.data.dtype not in (torch.float32, torch.float64):
        raise ValueError("device lognet needs an fp32/fp64 panel")
    dev = panel.device
    s = torch.cuda.current_stream().cuda_stream
    f64 = dict(dtype=torch.float64, device=dev)
    L = nlambda
    segs = np.stack([panel.seg_bounds[:, 0], panel.seg_bounds[:, 0] + panel.seg_nreal], 1)
    segs_t = torch.as_tensor(segs.astype(np.int64), device=dev)
    xc = torch.tensor(xcols, dtype=torch.int32, device=dev)
    vp_t = torch.tensor(vp, **f64)
    masks = np.ones((1 + K, K), dtype=np.uint8)
    for k in range(K):
        masks[1 + k, k] = 0
    masks_t = torch.from_numpy(masks).to(dev)
    nq = 1 + K
    a0 = torch.zeros((nq, L), **f64)
    beta = torch.zeros((nq, L, p), **f64)
    lam = torch.full((nq, L), float("nan"), **f64)
    devr = torch.zeros((nq, L), **f64)
    nlam = torch.zeros(nq, dtype=torch.int32, device=dev)
    npass = torch.zeros(nq, dtype=torch.int32, device=dev)
    dt = dtype_code(panel.data)
    X = panel.data
    off = lambda t: t.data_ptr() + t.element_size() * t.stride(0)
    if concurrent and L >= 3 and nq <= 256:
        # one launch: the full fit (problem 0) and the K fold fits run side by side, the
        # folds following the full fit's lambda sequence and stop through device flags
        progress = torch.zeros(2, dtype=torch.int32, device=dev)
        lampub = torch.zeros(L, **f64)
        _native.call("ate_lognet_path", dt, X.data_ptr(), panel.cm_ld, xc.data_ptr(), p, ycol,
                     segs_t.data_ptr(), K, masks_t.data_ptr(), nq, vp_t.data_ptr(), alpha,
                     flmin, thresh, maxit, 0, 0, L, a0.data_ptr(), beta.data_ptr(),
                     lam.data_ptr(), devr.data_ptr(), nlam.data_ptr(), npass.data_ptr(),
                     progress.data_ptr(), lampub.data_ptr(), s)
    else:
        # full problem: its own lambda sequence
        _native.call("ate_lognet_path", dt, X.data_ptr(), panel.cm_ld, xc.data_ptr(), p, ycol,
                     segs_t.data_ptr(), K, masks_t.data_ptr(), 1, vp_t.data_ptr(), alpha, flmin,
                     thresh, maxit, 0, 0, L, a0.data_ptr(), beta.data_ptr(), lam.data_ptr(),
                     devr.data_ptr(), nlam.data_ptr(), npass.data_ptr(), 0, 0, s)
        # fold problems on the full lambda sequence (count read on the device)
        _native.call("ate_lognet_path", dt, X.data_ptr(), panel.cm_ld, xc.data_ptr(), p, ycol,
                     segs_t.data_ptr(), K, off(masks_t), K, vp_t.data_ptr(), alpha, flmin,
                     thresh, maxit, lam.data_ptr(), nlam.data_ptr(), L, off(a0), off(beta),
                     off(lam), off(devr), nlam.data_ptr() + 4, npass.data_ptr() + 4, 0, 0, s)
    hold = torch.arange(K, dtype=torch.int32, device=dev)
    cvraw = torch.empty((K, L), **f64)
    _native.call("ate_lognet_cvloss", dt, X.data_ptr(), panel.cm_ld, xc.data_ptr(), p, ycol,
                 segs_t.data_ptr(), hold.data_ptr(), K, off(a0), off(beta),
                 nlam.data_ptr() + 4, L, cvraw.data_ptr(), s)
    fidx = torch.arange(K, dtype=torch.int32, device=dev)[None]
    nfold = torch.as_tensor(panel.seg_nreal.astype(np.float64), device=dev)[None]
    cvm = torch.empty((1, L), **f64)
    cvsd = torch.empty((1, L), **f64)
    sel = torch.empty((1, 2), dtype=torch.int32, device=dev)
    _native.call("ate_cv_select", cvraw.data_ptr(), fidx.data_ptr(), nfold.data_ptr(), K, 1,
                 nlam.data_ptr(), L, cvm.data_ptr(), cvsd.data_ptr(), sel.data_ptr(), None, 0,
                 s)
    coef = torch.cat([a0[0][:, None], beta[0]], 1)
    sl = sel[0].long()
    from .enet import poison_if_truncated
    cvm0, cvsd0, cmin, c1se = poison_if_truncated(npass[1:], cvm[0], cvsd[0], coef[sl[0]],
                                                  coef[sl[1]])
    return LognetCvResult(lam[0], nlam[:1], cvm0, cvsd0, sel[0], coef, cmin, c1se, npass)


def _cv_cpu(panel, xcols, ycol, vp, alpha, nlambda, flmin, thresh, maxit):
    X = panel.data.double()
    rows, fid = [], []
    for k, ((r0, _), nr) in enumerate(zip(panel.seg_bounds, panel.seg_nreal)):
        rows.append(np.arange(r0, r0 + nr))
        fid.append(np.full(nr, k))
    rows = np.concatenate(rows)
    fid = np.concatenate(fid)
    Xn = X[xcols][:, rows].T.numpy()
    yn = X[ycol][rows].numpy()
    cv = ref.cv_glmnet(Xn, yn, family="binomial", alpha=alpha, penalty_factor=vp, foldid=fid,
                       nlambda=nlambda, lambda_min_ratio=flmin, thresh=thresh, maxit=maxit)
    L = nlambda
    m = len(cv.lambdas)
    pad = lambda a: torch.as_tensor(np.r_[a, np.full(L - len(a), np.nan)])
    coef = np.column_stack([cv.fit.a0, cv.fit.beta])
    coef_t = torch.as_tensor(np.vstack([coef, np.full((L - m, coef.shape[1]), np.nan)]))
    sel = torch.tensor([cv.idx_min, cv.idx_1se], dtype=torch.int32)
    return LognetCvResult(pad(cv.lambdas), torch.tensor([m], dtype=torch.int32), pad(cv.cvm),
                          pad(cv.cvsd), sel, coef_t, coef_t[cv.idx_min], coef_t[cv.idx_1se],
                          torch.tensor([cv.fit.npasses]))
