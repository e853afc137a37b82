"""Exclusive prefix sums and stream compaction without inter-workgroup waiting
(csrc/scan.hip), for host loops that run beside other streams' kernels.

torch.cumsum / torch.nonzero on a GPU run rocprim's single-pass decoupled-lookback
kernels, whose workgroups spin until their predecessors publish; with several forests
grown side by side (estimators/crossfit.py) the config-3 shard stalled for 33 s with such
kernels resident on two streams (profiles/r03_cfg3b). These three-launch scans never wait
on another workgroup. CPU tensors use torch.
"""
from __future__ import annotations

import torch

from .. import _native


def exclusive_cumsum(x: torch.Tensor, total: bool = False):
    """out[i] = sum(x[:i]) of a 1-D int32 / int64 tensor (same dtype); with total=True
    returns (out, tot) where tot is a [1] tensor holding sum(x), still on the device."""
    if x.dtype not in (torch.int32, torch.int64) or x.dim() != 1:
        raise TypeError("exclusive_cumsum: 1-D int32 or int64 tensor")
    if not x.is_cuda:
        inc = torch.cumsum(x, 0, dtype=x.dtype)
        out = inc - x
        return (out, inc[-1:].clone() if x.numel() else torch.zeros(1, dtype=x.dtype)) \
            if total else out
    x = x.contiguous()
    n = x.numel()
    out = torch.empty_like(x)
    tot = torch.zeros(1, dtype=x.dtype, device=x.device)
    if n:
        part = torch.empty(int(_native.hip().ate_scan_parts(n)), dtype=x.dtype, device=x.device)
        name = "ate_excl_scan_i32" if x.dtype == torch.int32 else "ate_excl_scan_i64"
        _native.call(name, x.data_ptr(), n, out.data_ptr(), part.data_ptr(), tot.data_ptr(),
                     torch.cuda.current_stream(x.device).cuda_stream)
    return (out, tot) if total else out


def compact_rows(mask: torch.Tensor) -> torch.Tensor:
    """Ascending indices of the True entries of a 1-D bool tensor (torch.nonzero(mask)
    without the lookback kernel). One host sync for the count."""
    if not mask.is_cuda:
        return torch.nonzero(mask).flatten()
    n = mask.numel()
    flags = mask.to(torch.int32) if n < 2 ** 31 else mask.to(torch.int64)
    pos, tot = exclusive_cumsum(flags, total=True)
    m = int(tot.item())
    out = torch.empty(m + 1, dtype=torch.int64, device=mask.device)
    dest = torch.where(mask, pos.long(), torch.full_like(pos, m, dtype=torch.int64))
    out.scatter_(0, dest, torch.arange(n, device=mask.device))
    return out[:m]
