"""K02 column moments / R ``scale()`` and K21 interaction expansion (csrc/prep.hip).

Device tensors run the HIP kernels (no fallback: a missing library raises); CPU
tensors use the same formulas in float64 torch.
"""
from __future__ import annotations

import torch

from .. import _native

CHUNKS = 64


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _colmajor(X: torch.Tensor) -> torch.Tensor:
    """[n, p] float64 -> contiguous column-major storage as a [p, n] tensor."""
    return X.double().t().contiguous()


def col_moments(X: torch.Tensor) -> torch.Tensor:
    """[n, p] -> [p, 3] float64 = (non-NaN count, mean, sample SD) per column, the
    statistics R's ``scale()`` uses (NaNs ignored)."""
    n, p = X.shape
    if not X.is_cuda:
        x = X.double()
        ok = ~torch.isnan(x)
        cnt = ok.sum(0).double()
        mean = torch.where(ok, x, 0.0).sum(0) / cnt
        dev = torch.where(ok, x - mean, 0.0)
        sd = torch.sqrt((dev * dev).sum(0) / (cnt - 1))
        return torch.stack([cnt, mean, sd], 1)
    Xc = _colmajor(X)
    part = torch.empty(p * CHUNKS * 2, dtype=torch.float64, device=X.device)
    mean = torch.empty(p, dtype=torch.float64, device=X.device)
    mom = torch.empty((p, 3), dtype=torch.float64, device=X.device)
    _native.call("ate_col_moments", Xc.data_ptr(), n, n, p, part.data_ptr(), mean.data_ptr(),
                 mom.data_ptr(), _stream())
    return mom


def r_scale(X: torch.Tensor, cols=None, constant_to_one: bool = False) -> torch.Tensor:
    """R ``scale()`` of the selected columns (default all): centre, divide by the
    sample SD; returns a new [n, p] float64 tensor. ``constant_to_one`` divides
    zero-SD columns by 1 instead of producing NaN (the CSV loader's guard)."""
    n, p = X.shape
    sel = torch.zeros(p, dtype=torch.uint8)
    sel[list(range(p)) if cols is None else list(cols)] = 1
    mom = col_moments(X)
    if constant_to_one:
        mom[:, 2] = torch.where(mom[:, 2] > 0, mom[:, 2], torch.ones_like(mom[:, 2]))
    if not X.is_cuda:
        x = X.double().clone()
        m = sel.bool()
        x[:, m] = (x[:, m] - mom[m, 1]) / mom[m, 2]
        return x
    Xc = _colmajor(X)
    s = sel.to(X.device)
    _native.call("ate_standardize", Xc.data_ptr(), n, n, p, mom.data_ptr(), s.data_ptr(),
                 _stream())
    return Xc.t()


def interactions(X: torch.Tensor) -> torch.Tensor:
    """K21: [x, x_c1 * x_c2 for all ordered pairs incl. squares] -> [n, p + p^2]
    (belloni's design, quirk Q10)."""
    n, p = X.shape
    if not X.is_cuda:
        x = X.double()
        return torch.cat([x, (x[:, :, None] * x[:, None, :]).reshape(n, p * p)], 1)
    Xc = _colmajor(X)
    out = torch.empty((p + p * p, n), dtype=torch.float64, device=X.device)
    _native.call("ate_interactions", Xc.data_ptr(), n, n, p, out.data_ptr(), n, _stream())
    return out.t()
