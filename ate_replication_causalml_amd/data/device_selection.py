"""Device selection-bias transform (K04 select_compact; csrc/select.hip).

Same semantics as data/selection.py (first round(pt*k) candidates per arm in row
order, quirk Q17 under compat="reference"), for panels that live in HBM (1e8 rows):
returns the kept row indices in order. CPU tensors use the host implementation.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _native
from .selection import drop_indices

_COLS = ("g2000", "g2002", "p2000", "p2002", "p2004", "city", "yob")


def keep_indices(X, W, names, pt=0.85, pc=0.85, compat="reference", device=None) -> torch.Tensor:
    dev = torch.device(device) if device is not None else (
        X.device if isinstance(X, torch.Tensor) else torch.device("cpu"))
    if dev.type != "cuda":
        Xn = X.cpu().numpy() if isinstance(X, torch.Tensor) else np.asarray(X)
        Wn = W.cpu().numpy() if isinstance(W, torch.Tensor) else np.asarray(W)
        drop = drop_indices(Xn, Wn, list(names), pt, pc, compat)
        keep = np.ones(len(Wn), dtype=bool)
        keep[drop] = False
        return torch.from_numpy(np.flatnonzero(keep))
    Xt = torch.as_tensor(X, dtype=torch.float64, device=dev).T.contiguous()   # [p][n]
    Wt = torch.as_tensor(W, dtype=torch.float64, device=dev).contiguous()
    n = Wt.numel()
    idx = {nm: i for i, nm in enumerate(names)}
    last = "p2002" if compat == "reference" else "p2004"
    cols = torch.tensor([idx[c] for c in _COLS] + [idx[last]], dtype=torch.int32, device=dev)
    nblk = (n + 255) // 256
    flags = torch.empty(n, dtype=torch.uint8, device=dev)
    keep = torch.empty(n, dtype=torch.uint8, device=dev)
    scratch = torch.zeros(3 * nblk + 4, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    _native.call("ate_select_compact", Xt.data_ptr(), n, Wt.data_ptr(), cols.data_ptr(), pt, pc,
                 flags.data_ptr(), keep.data_ptr(), scratch.data_ptr(), out.data_ptr(),
                 torch.cuda.current_stream().cuda_stream)
    total = int(scratch[3 * nblk + 2].item())
    return out[:total]
