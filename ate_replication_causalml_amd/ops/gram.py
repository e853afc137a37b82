"""K01 Gram op: per-segment G_s = X_s' diag(w) X_s (fp64 output [nseg, P, P]).

GPU: ``csrc/gram.hip`` (bf16 MFMA 16x16x32 for bf16 panels; fp32 / fp64 MFMA
16x16x4 for fp32 / fp64 panels, optional row weights). CPU: float64 torch.
Launch geometry (tiles, row chunks) is computed here once per panel shape and
cached together with the slab workspace so repeated calls (IRLS iterations,
graph capture) allocate nothing.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .. import _native
from .panel import DevicePanel

BF16_TILE, BF16_K = 128, 64
BF16_TILE_BIG = 256
SMALL_TILE, SMALL_K = 64, 16
TARGET_WG = 2048   # workgroups per launch (>= 8 per CU on 256 CUs)

# 256-tile kernel: 1 = 2-stage BK=64 LDS-DMA (default), 0 = 4-stage BK=32 pipeline.
# Measured at N=1e7, p=500 (tools/gram_only.py, tools/pmc_gram.sh): 4.0 vs 5.0 ms -- the
# BK=32 stages fetch half cache lines (TA busy 3x, L2 requests 2x) and lose more than the
# deeper prefetch gains.
GRAM_VARIANT = int(os.environ.get("ATE_GRAM_VARIANT", "1"))

_plan_cache = {}


def _stream():
    return torch.cuda.current_stream().cuda_stream


class GramPlan:
    def __init__(self, panel: DevicePanel, weighted: bool):
        bf16 = panel.dtype == torch.bfloat16
        if bf16 and weighted:
            raise ValueError("weighted Gram needs an fp32/fp64 panel")
        P = panel.P
        if bf16:
            T = BF16_TILE_BIG if P % BF16_TILE_BIG == 0 else BF16_TILE
        else:
            T = SMALL_TILE
        K = BF16_K if bf16 else SMALL_K
        if P % T:
            raise ValueError(f"panel P={P} must be a multiple of {T}")
        nt = P // T
        tiles = [(a, b) for a in range(nt) for b in range(a, nt)]
        ntiles = len(tiles)
        rows_total = int((panel.seg_bounds[:, 1] - panel.seg_bounds[:, 0]).sum())
        # 256-tile: 1 WG (128 KB LDS) per CU; ~12 short-lived WGs per CU keep the three tiles
        # of a row chunk close in time so their shared panels are L2 hits (measured 4.65 ->
        # 4.09 ms at N=1e7, p=500 going from 768 to 3072 WGs)
        target = 3072 if T == BF16_TILE_BIG else TARGET_WG
        target = int(os.environ.get("ATE_GRAM_WG", target))
        nchunk_target = max(1, target // ntiles)
        ch_rows = max(K, (rows_total // nchunk_target) // K * K)
        chunks = []
        seg_chunk0 = [0]
        for s, (r0, r1) in enumerate(panel.seg_bounds):
            r = int(r0)
            while r < r1:
                e = min(int(r1), r + ch_rows)
                chunks.append((r, e, s, 0))
                r = e
            seg_chunk0.append(len(chunks))
        dev = panel.device
        self.T, self.K, self.ntiles, self.nchunks = T, K, ntiles, len(chunks)
        self.tiles = torch.tensor(tiles, dtype=torch.int32, device=dev)
        ch = np.zeros(len(chunks), dtype=[("r0", "<i8"), ("r1", "<i8"), ("seg", "<i4"),
                                          ("pad", "<i4")])
        for i, c in enumerate(chunks):
            ch[i] = c
        self.chunks = torch.from_numpy(ch.view(np.uint8).copy()).to(dev)
        self.seg_chunk0 = torch.tensor(seg_chunk0, dtype=torch.int32, device=dev)
        slab_dtype = torch.float32 if panel.dtype != torch.float64 else torch.float64
        self.slab = torch.empty(self.nchunks * ntiles * T * T, dtype=slab_dtype, device=dev)
        self.G = torch.empty((panel.nseg, P, P), dtype=torch.float64, device=dev)


def plan_for(panel: DevicePanel, weighted=False) -> GramPlan:
    key = (panel.data.data_ptr(), tuple(panel.data.shape), panel.data.dtype, weighted,
           tuple(map(tuple, panel.seg_bounds)))
    pl = _plan_cache.get(key)
    if pl is None:
        pl = GramPlan(panel, weighted)
        _plan_cache[key] = pl
    return pl


def gram(panel: DevicePanel, w: torch.Tensor | None = None, done: torch.Tensor | None = None,
         out: torch.Tensor | None = None) -> torch.Tensor:
    """Per-segment Gram stack [nseg, P, P] (fp64). ``w``: optional row weights (panel order)."""
    X = panel.data
    if not X.is_cuda:
        return _gram_cpu(panel, w, out)
    pl = plan_for(panel, weighted=w is not None)
    G = pl.G if out is None else out
    s = _stream()
    if X.dtype == torch.bfloat16:
        _native.call("ate_gram_bf16", X.data_ptr(), panel.ld, panel.P, pl.T, GRAM_VARIANT,
                     pl.tiles.data_ptr(),
                     pl.ntiles, pl.chunks.data_ptr(), pl.nchunks, pl.seg_chunk0.data_ptr(),
                     panel.nseg, pl.slab.data_ptr(), G.data_ptr(), s)
    else:
        name = "ate_gram_f64" if X.dtype == torch.float64 else "ate_gram_f32"
        if w is not None:
            assert w.dtype == X.dtype and w.numel() == panel.ld
        _native.call(name, X.data_ptr(), panel.ld, panel.P, 0 if w is None else w.data_ptr(),
                     pl.tiles.data_ptr(), pl.ntiles, pl.chunks.data_ptr(), pl.nchunks,
                     pl.seg_chunk0.data_ptr(), panel.nseg, pl.slab.data_ptr(), G.data_ptr(),
                     0 if done is None else done.data_ptr(), s)
    return G


def _gram_cpu(panel, w, out):
    X = panel.data.double()
    Gs = []
    for (r0, r1) in panel.seg_bounds:
        Xs = X[:, r0:r1]
        A = Xs if w is None else Xs * w[r0:r1].double()
        Gs.append(A @ Xs.T)
    G = torch.stack(Gs)
    if out is not None:
        out.copy_(G)
        return out
    return G


def gram_reference(panel: DevicePanel, w=None) -> torch.Tensor:
    """Plain fp64 PyTorch reference of the same op (for numerics tests)."""
    X = panel.data.double().cpu()
    wv = None if w is None else w.double().cpu()
    out = []
    for (r0, r1) in panel.seg_bounds:
        Xs = X[:, r0:r1]
        A = Xs if wv is None else Xs * wv[r0:r1]
        out.append(A @ Xs.T)
    return torch.stack(out)
