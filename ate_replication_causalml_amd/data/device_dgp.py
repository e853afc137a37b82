"""Synthetic tutorial-shape panels generated directly on the device (K-fold,
row-sharded across ranks) for the scaled configs (N = 1e6 .. 1e8, p = 21 .. 2000).

Global row g belongs to fold ``g * K // N``; rank r of R holds the r-th contiguous
slice of every fold. Rows are a pure function of (seed, g) (``csrc/dgp.hip``), so
the union of all shards is the same data set for every world size.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _native
from ..ops.panel import DevicePanel, empty_panel, dtype_code
from . import dgp as host_dgp

N_TUTORIAL_COLS = 21


def fold_slices(n_total: int, folds: int, rank: int = 0, world: int = 1, align: int = 0):
    """[(global_start, count)] of this rank's slice of each fold. ``align`` > 0: slices are
    cut at multiples of ``align`` rows from the fold start (whole blocks per rank), the
    layout of the world-size-invariant exact reduction mode (ops/gram.py ``exact``)."""
    out = []
    for k in range(folds):
        f0, f1 = k * n_total // folds, (k + 1) * n_total // folds
        m = f1 - f0
        if align:
            nb = -(-m // align)
            a = min(f1, f0 + (rank * nb // world) * align)
            b = min(f1, f0 + ((rank + 1) * nb // world) * align)
        else:
            a = f0 + rank * m // world
            b = f0 + (rank + 1) * m // world
        out.append((a, b - a))
    return out


def synthetic_panel(n_total: int, p: int = 500, folds: int = 5, seed: int = 1991,
                    dtype: str = "bf16", device="cpu", rank: int = 0, world: int = 1,
                    blocked: bool = False, align: int = 0) -> DevicePanel:
    """``align`` > 0: block-aligned rank slices (fold_slices); the panel then records
    ``exact_block`` = align, the row block of the exact (world-size-invariant) Gram."""
    if p < N_TUTORIAL_COLS:
        raise ValueError("p must be >= 21 (tutorial columns)")
    p_extra = p - N_TUTORIAL_COLS
    slices = fold_slices(n_total, folds, rank, world, align)
    hi_lo = dtype == "bf16"
    names = ["one"] + [f"x{j}" for j in range(p)] + ["W", "Y"]
    if hi_lo:
        names += ["W_hi", "W_lo", "Y_hi", "Y_lo"]
    cpad = 128 if dtype == "bf16" else 64
    P = (len(names) + cpad - 1) // cpad * cpad
    pan = empty_panel([c for _, c in slices], P, dtype=dtype, device=device, blocked=blocked)
    pan.cols = {nm: i for i, nm in enumerate(names)}
    pan.xcols = [pan.cols[f"x{j}"] for j in range(p)]
    # global row ids of this shard (panel order)
    rid = torch.full((pan.ld,), -1, dtype=torch.int64, device=device)
    for (g0, cnt), (r0, _) in zip(slices, pan.seg_bounds):
        rid[r0:r0 + cnt] = torch.arange(g0, g0 + cnt, device=device)
    pan.row_index = rid
    pan.identity = len(slices) == 1 and slices[0][0] == 0
    if pan.data.is_cuda:
        s = torch.cuda.current_stream().cuda_stream
        for (g0, cnt), (r0, _) in zip(slices, pan.seg_bounds):
            _native.call("ate_dgp_fill", dtype_code(pan.data), pan.data.data_ptr(),
                         *pan.strides(), int(r0), cnt, g0, seed, p_extra, int(hi_lo), s)
    else:
        cm = torch.zeros((pan.P, pan.ld), dtype=pan.data.dtype) if blocked else pan.data
        for (g0, cnt), (r0, _) in zip(slices, pan.seg_bounds):
            cts, binc, extra, W, Y, _ = host_dgp.raw_columns(cnt, seed, p_extra, row_offset=g0)
            cols = [np.ones(cnt), *cts.T, *binc.T, *extra.T, W, Y]
            if hi_lo:
                cols += [W, np.zeros(cnt), Y, np.zeros(cnt)]
            block = torch.from_numpy(np.stack(cols)).to(pan.data.dtype)
            cm[:block.shape[0], r0:r0 + cnt] = block
        if blocked:
            pan.data.copy_(cm.reshape(pan.P, -1, 64).permute(1, 0, 2))
    pan.n = sum(c for _, c in slices)
    pan.exact_block = int(align)
    return pan
