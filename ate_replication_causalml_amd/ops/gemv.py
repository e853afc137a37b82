"""Grouped panel GEMVs (csrc/panel_ops.hip) with host fallbacks.

xtv(panel, cols, v, grp, A) -> [A, len(cols)]: per-group X' v over the panel rows.
xv(panel, cols, V, grp)     -> [ld]: row i gets X_i . V[grp[i]] (0 where grp < 0).
"""
from __future__ import annotations

import torch

from .. import _native
from .devconst import const
from .panel import dtype_code


def _cols(panel, cols):
    # cached device constant: no host->device copy per call (hipGraph-capturable)
    return const(list(cols), torch.int32, panel.device)


def xtv(panel, cols, v: torch.Tensor, grp: torch.Tensor, A: int) -> torch.Tensor:
    X = panel.data
    if not X.is_cuda:
        M = X[list(cols)].double()
        return torch.stack([M @ torch.where(grp == a, v, torch.zeros_like(v)) for a in range(A)])
    out = torch.empty((A, len(cols)), dtype=torch.float64, device=X.device)
    c = _cols(panel, cols)
    _native.call("ate_panel_xtv", dtype_code(X), X.data_ptr(), panel.cm_ld, c.data_ptr(), len(cols),
                 v.contiguous().data_ptr(), grp.data_ptr(), panel.ld, A, out.data_ptr(),
                 torch.cuda.current_stream().cuda_stream)
    return out


def xv(panel, cols, V: torch.Tensor, grp: torch.Tensor) -> torch.Tensor:
    X = panel.data
    if not X.is_cuda:
        M = X[list(cols)].double()
        full = V.double() @ M                            # [A, ld]
        g = grp.long()
        out = full.gather(0, g.clamp(min=0)[None])[0]
        return torch.where(g >= 0, out, torch.zeros_like(out))
    out = torch.empty(panel.ld, dtype=torch.float64, device=X.device)
    c = _cols(panel, cols)
    _native.call("ate_panel_xv", dtype_code(X), X.data_ptr(), panel.cm_ld, c.data_ptr(), len(cols),
                 V.contiguous().double().data_ptr(), V.shape[0], grp.data_ptr(), panel.ld,
                 out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    return out
