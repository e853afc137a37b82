"""K01 Gram op: per-segment G_s = X_s' diag(w) X_s (fp64 output [nseg, P, P]).

GPU: ``csrc/gram.hip`` (bf16 MFMA 16x16x32 for bf16 panels; fp32 / fp64 MFMA
16x16x4 for fp32 / fp64 panels, optional row weights). CPU: float64 torch.
Launch geometry (tiles, row chunks) is computed here once per panel shape and
cached together with the slab workspace so repeated calls (IRLS iterations,
graph capture) allocate nothing.
"""
from __future__ import annotations

import contextlib
import os

import numpy as np
import torch

from .. import _native
from ..utils.graphs import pin
from .panel import DevicePanel

BF16_TILE, BF16_K = 128, 64
BF16_TILE_BIG = 256
SMALL_TILE, SMALL_K = 64, 16
TARGET_WG = 2048   # workgroups per launch (>= 8 per CU on 256 CUs)

# bf16 kernel for P % 512 == 0: "pair" (symmetry-aware paired tiles, default) or "tile256"
# (three full 256 tiles per 512 columns). For P % 256 == 0 otherwise: tile256; else 128.
# (A 4-stage BK=32 variant of tile256 measured 5.0 vs 4.0 ms and was dropped: BK=32
# stages fetch half cache lines; profiles/r01_pmc/gram_variant*.txt.)
GRAM_KERNEL = os.environ.get("ATE_GRAM_KERNEL", "pair")
PAIR_SLOTS = 272
# P == 512 (p <= 505 covariates, the bench shape): ATE_GRAM_TRI=1 selects the split-triangle
# kernel (csrc/gram.hip gram_bf16_tri_kernel: 864 instead of 1024 column reads per chunk).
# Measured and NOT the default (profiles/r06_gram): equal to the paired-tile kernel alone
# (2.54-2.56 vs 2.52-2.56 ms) and 0.45 ms slower inside the single ate_dml call (2.73 vs 2.29)
TRI_SLOTS, TRI_SPLIT = 288, 22
GRAM_TRI = os.environ.get("ATE_GRAM_TRI", "0") == "1"
# Panels that carry one-byte copies of their {0, 1} columns (DevicePanel.bytes8: physical
# columns 384..511 of a P = 512 blocked bf16 panel) stream those to the paired-tile Gram as
# bytes (csrc/gram.hip): 896 instead of 1,024 bytes per row, the same Gram bits.
# ATE_GRAM_BYTES=0 reads them as bf16 (A/B).
BYTE_COLS = os.environ.get("ATE_GRAM_BYTES", "1") == "1"
PLAN_CACHE_MAX = int(os.environ.get("ATE_GRAM_PLAN_CACHE", 8))

_plan_cache: dict = {}
_slot = 0


@contextlib.contextmanager
def plan_slot(i: int):
    """Plans (slab + Gram output buffers) made inside this context are private to slot ``i``,
    so independent estimator calls captured in separate hipGraphs can be in flight on
    separate streams at once without sharing a workspace (bench.py --inflight)."""
    global _slot
    prev, _slot = _slot, int(i)
    try:
        yield
    finally:
        _slot = prev


def _stream():
    return torch.cuda.current_stream().cuda_stream


class GramPlan:
    def __init__(self, panel: DevicePanel, weighted: bool, exact: bool = False):
        bf16 = panel.dtype == torch.bfloat16
        if bf16 and weighted:
            raise ValueError("weighted Gram needs an fp32/fp64 panel")
        P = panel.P
        self.pair = bf16 and P % (2 * BF16_TILE_BIG) == 0 and GRAM_KERNEL == "pair"
        self.tri = self.pair and P == 512 and GRAM_TRI
        if bf16:
            T = BF16_TILE_BIG if P % BF16_TILE_BIG == 0 else BF16_TILE
        else:
            T = SMALL_TILE
        K = BF16_K if bf16 else SMALL_K
        if P % T:
            raise ValueError(f"panel P={P} must be a multiple of {T}")
        nt = P // T
        if self.tri:
            tiles, blocks = [(0, 0, 0, 0), (0, 0, 1, 0)], tri_blocks()
        elif self.pair:
            tiles, blocks = _pair_tiles(nt, bal=bool(_native.hip().ate_gram_pair_bal()))
        else:
            tiles = [(a, b) for a in range(nt) for b in range(a, nt)]
        ntiles = len(tiles)
        rows_total = int((panel.seg_bounds[:, 1] - panel.seg_bounds[:, 0]).sum())
        # 256-tile / pair: 1 WG (128 KB LDS) per CU; ~12 short-lived WGs per CU keep the three tiles
        # of a row chunk close in time so their shared panels are L2 hits (measured 4.65 ->
        # 4.09 ms at N=1e7, p=500 going from 768 to 3072 WGs)
        target = 3072 if T == BF16_TILE_BIG else TARGET_WG
        whole_rounds = False
        if self.pair:
            # one Gram alone on the chip: 5 whole rounds of workgroups (N=1e7, p=500, 5 folds:
            # 2.48 ms vs 2.61 at 2040 WGs and 2.70 at 2060, profiles/r02c_gram; ATE_GRAM_ROUNDS
            # overrides the round count for sweeps); bench.py's
            # overlapped fits set ATE_GRAM_PAIR_WG (finer workgroups share CUs with path solves)
            env = os.environ.get("ATE_GRAM_PAIR_WG")
            whole_rounds = env is None
            rounds = int(os.environ.get("ATE_GRAM_ROUNDS", "5"))
            target = int(env) if env is not None else rounds * _cu_count(panel.device)
        target = int(os.environ.get("ATE_GRAM_WG", target))
        nchunk_target = max(1, target // ntiles)
        chunks = []
        seg_chunk0 = [0]
        if exact:
            # one chunk per row block of the segment (blocks counted from the segment start:
            # the same global blocks at every world size, data/device_dgp.fold_slices(align))
            B = int(panel.exact_block)
            if B <= 0 or B % K:
                raise ValueError("exact Gram needs a block-aligned panel (synthetic_panel("
                                 f"align=B) with B a multiple of {K})")
            for s_, (r0, r1) in enumerate(panel.seg_bounds):
                r = int(r0)
                while r < r1:
                    e = min(int(r1), r + B)
                    chunks.append((r, e, s_, 0))
                    r = e
                seg_chunk0.append(len(chunks))
        elif self.pair:
            # equal chunks, the same count in every segment, total workgroups <= target: a
            # launch of 2 x nseg x k near-equal workgroups fills whole rounds of CUs instead of
            # leaving a few stragglers of a ~0.3 ms workgroup to run alone at the end (2060 WGs
            # on 256 CUs = 8 rounds + 12 WGs before this)
            chunks, seg_chunk0 = pair_chunks(panel.seg_bounds, K, ntiles, target,
                                             _cu_count(panel.device) if whole_rounds else 0)
        else:
            ch_rows = max(K, (rows_total // nchunk_target) // K * K)
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
        if self.pair:
            self.blocks = torch.tensor(blocks, dtype=torch.int32, device=dev)
        ch = np.zeros(len(chunks), dtype=[("r0", "<i8"), ("r1", "<i8"), ("seg", "<i4"),
                                          ("pad", "<i4")])
        for i, c in enumerate(chunks):
            ch[i] = c
        self.chunks = torch.from_numpy(ch.view(np.uint8).copy()).to(dev)
        self.seg_chunk0 = torch.tensor(seg_chunk0, dtype=torch.int32, device=dev)
        slab_dtype = torch.float32 if panel.dtype != torch.float64 else torch.float64
        per_tile = (TRI_SLOTS if self.tri else PAIR_SLOTS) * 256 if self.pair else T * T
        self.slab = torch.empty(self.nchunks * ntiles * per_tile, dtype=slab_dtype, device=dev)
        self.G = torch.empty((panel.nseg, P, P), dtype=torch.float64, device=dev)
        self.Gx = torch.empty((2, panel.nseg, P, P), dtype=torch.int64, device=dev) \
            if exact else None


def pair_chunks(seg_bounds, K: int, ntiles: int, target: int, ncu: int = 0):
    """Row chunks of the paired-tile Gram: every segment cut into the same number k of
    near-equal chunks (multiples of the K-step; the last one ends at the segment end), with
    ntiles x nseg x k <= target workgroups. ncu > 0: lower k (by at most half) until the
    launch is a whole number of rounds of ncu workgroups. Returns (chunks [(r0, r1, seg, 0)],
    seg_chunk0 [nseg + 1])."""
    nseg = max(1, len(seg_bounds))
    k = max(1, max(1, target // ntiles) // nseg)
    if ncu > 0:
        per = ntiles * nseg
        kr = k
        while kr > 1 and (per * kr) % ncu:
            kr -= 1
        if (per * kr) % ncu == 0 and 2 * kr >= k:
            k = kr
    chunks, seg_chunk0 = [], [0]
    for s, (r0, r1) in enumerate(seg_bounds):
        r0, r1 = int(r0), int(r1)
        steps = (r1 - r0) // K
        ks = max(1, min(k, steps))
        for j in range(ks):
            a = r0 + (steps * j // ks) * K
            e = r0 + (steps * (j + 1) // ks) * K if j + 1 < ks else r1
            chunks.append((a, e, s, 0))
        seg_chunk0.append(len(chunks))
    return chunks, seg_chunk0


def _cu_count(dev) -> int:
    try:
        return int(torch.cuda.get_device_properties(dev).multi_processor_count)
    except Exception:  # noqa: BLE001 - CPU / no device: MI355X has 256 CUs
        return 256


def _pair_tiles(nt: int, bal: bool = True):
    """Tile list (a, b, type, 0) and slab block table for the paired-tile kernel
    (csrc/gram.hip gram_bf16_pair_kernel): every diagonal pair (a, b) follows the
    off-diagonal tile (a, b) that streams the same columns; remaining off-diagonal tiles
    after. Returns (tiles, blocks[ntiles][PAIR_SLOTS] of 16-column block (I, J)).
    ``bal`` (the library's GRAM_BAL, ate_gram_pair_bal): in a diagonal pair every wave holds
    34 blocks -- each triangle wave's last two, (6, 7) and (7, 7) of its triangle, are
    computed by the rectangle wave of the same region and half."""
    tiles = []
    for a in range(0, nt - 1, 2):
        tiles.append((a, a + 1, 0, 0))
        tiles.append((a, a + 1, 1, 0))
    if nt % 2:
        tiles.append((nt - 1, nt - 1, 2, 0))
    paired = {(a, a + 1) for a in range(0, nt - 1, 2)}
    tiles += [(a, b, 0, 0) for a in range(nt) for b in range(a + 1, nt) if (a, b) not in paired]
    blocks = []
    for (a, b, typ, _) in tiles:
        tb = [(-1, -1)] * PAIR_SLOTS
        if typ == 0:
            for w in range(8):
                wr, wc = w >> 2, w & 3
                for m in range(8):
                    for n in range(4):
                        tb[w * 32 + m * 4 + n] = (a * 16 + wr * 8 + m, b * 16 + wc * 4 + n)
        else:
            rs, ts = (34, 34) if bal else (32, 36)     # blocks per rectangle / triangle wave
            for w in range(4):                         # rectangles rows 0-7 x cols 8-15
                region, half = w >> 1, w & 1
                if typ == 2 and region == 1:
                    continue
                base = (a if region == 0 else b) * 16
                for m in range(8):
                    for n in range(4):
                        tb[w * rs + m * 4 + n] = (base + m, base + 8 + half * 4 + n)
                if bal:                                # the triangle's (6, 7), (7, 7)
                    t0 = base + half * 8
                    tb[w * rs + 32] = (t0 + 6, t0 + 7)
                    tb[w * rs + 33] = (t0 + 7, t0 + 7)
            for w in range(4):                         # triangles I <= J in 0-7 / 8-15
                region, half = w >> 1, w & 1
                if typ == 2 and region == 1:
                    continue
                base = (a if region == 0 else b) * 16 + half * 8
                idx = 0
                for m in range(8):
                    for n in range(m, 8):
                        if idx < ts:
                            tb[4 * rs + w * ts + idx] = (base + m, base + n)
                        idx += 1
        blocks.append(tb)
    return tiles, blocks


def tri_roles():
    """Wave roles of the split-triangle kernel (csrc/gram.hip gram_bf16_tri_kernel, same
    order): per workgroup type, per wave, (fragment column blocks, block list as pairs of
    fragment indices). Mirrors RoleRect / RoleTri / RoleMix."""
    def rect(a0, na, b0, nb):
        return ([a0 + f for f in range(na)] + [b0 + f for f in range(nb)],
                [(m, na + n) for m in range(na) for n in range(nb)])

    def tri(s0, s):
        return [s0 + f for f in range(s)], [(m, n) for m in range(s) for n in range(m, s)]
    mix_blocks = [(0, n) for n in range(1, 6)] + [
        (1 + 5 * g + m, 1 + 5 * g + n) for g in range(2) for m in range(5) for n in range(m, 5)]
    t0 = [tri(0, 8), tri(8, 8), rect(0, 4, 8, 8), rect(4, 4, 8, 8), rect(0, 6, 16, 6),
          rect(6, 5, 16, 6), rect(11, 5, 16, 6), tri(16, 6)]
    t1 = [rect(0, 7, 22, 5), rect(7, 7, 22, 5), rect(14, 7, 22, 5), rect(0, 7, 27, 5),
          rect(7, 7, 27, 5), rect(14, 7, 27, 5), rect(21, 6, 27, 5),
          ([21 + f for f in range(11)], mix_blocks)]
    return [t0, t1]


def tri_blocks():
    """Slab block table [2][TRI_SLOTS] of 16-column Gram blocks (I, J) for the
    split-triangle kernel: wave w of a workgroup writes its k-th block to slot 36 w + k."""
    out = []
    for roles in tri_roles():
        tb = [(-1, -1)] * TRI_SLOTS
        for w, (fc, bl) in enumerate(roles):
            assert len(bl) <= 36
            for k, (a, b) in enumerate(bl):
                tb[w * 36 + k] = (fc[a], fc[b])
        out.append(tb)
    return out


def plan_for(panel: DevicePanel, weighted=False, exact=False) -> GramPlan:
    """Cached launch plan + workspace. The cache is an LRU of ``PLAN_CACHE_MAX`` entries
    (a bf16 plan at N=1e7 holds ~0.5 GB of slab): evicting drops only the cache's
    reference, and a hipGraph that captured the plan keeps it alive (utils/graphs.pin).
    Keyed by the panel's address too: the plan owns the returned Gram buffer, and two
    live panels of one shape must not share it."""
    key = (panel.data.data_ptr(), tuple(panel.data.shape), panel.data.dtype, weighted,
           tuple(map(tuple, panel.seg_bounds)), _slot, exact)
    pl = _plan_cache.pop(key, None)
    if pl is None:
        while len(_plan_cache) >= PLAN_CACHE_MAX:
            _plan_cache.pop(next(iter(_plan_cache)))
        pl = GramPlan(panel, weighted, exact)
    _plan_cache[key] = pl          # most recently used last
    return pin(pl)


def clear_plans():
    """Drop every cached Gram plan (graphs that captured one keep theirs alive)."""
    _plan_cache.clear()


_STAGES = {"all": 3, "tiles": 1, "reduce": 2}


EXACT_LIMB_BOUND = 2.0 ** 38   # |Gram entry| bound of the fixed 2^24-scale int64 limbs


def check_exact_range(panel: DevicePanel, n_total: int | None = None, w=None, comm=None):
    """Raise if the exact mode's fixed-scale limbs could wrap: the hi limb of an entry is
    floor(v 2^24) summed over chunks in int64, exact only while every |G_jk| < 2^38, and
    |G_jk| <= max_i |x_ij| max_i |x_ik| * n_total (weighted: times max |w|). ``n_total``:
    rows over ALL ranks (weak scaling grows it). One reduction over the panel; skipped
    inside a graph capture (the guard runs on the eager first call of a layout).

    ``comm`` (world > 1): the max |x| (and max |w|) are all-reduced first, so every rank
    takes the same decision -- a rank that raised alone would leave its peers blocked in
    the limb all-reduce. Call it where every rank runs it eagerly (estimators/lasso.py
    dml_phases does, once per layout)."""
    X = panel.data
    if X.is_cuda and torch.cuda.is_current_stream_capturing():
        return
    dims = (0, 2) if panel.blocked else 1                 # no |X| temporary of the panel
    amax = torch.maximum(X.amax(dim=dims), -X.amin(dim=dims)).double()
    m = torch.stack([amax.max(), w.abs().max().double() if w is not None
                     else torch.ones((), dtype=torch.float64, device=amax.device)])
    if comm is not None and comm.world_size > 1:
        comm.all_reduce_max_(m)
    xm, wm = (float(v) for v in m.cpu())
    bound = xm ** 2 * float(n_total or panel.n)
    if w is not None:
        bound *= wm
    if not bound < EXACT_LIMB_BOUND:
        raise ValueError(f"exact Gram: entries up to {bound:.3g} exceed the int64 limb range "
                         f"(2^38 = {EXACT_LIMB_BOUND:.3g}); rescale the columns or use the "
                         "non-exact mode")


def gram(panel: DevicePanel, w: torch.Tensor | None = None, done: torch.Tensor | None = None,
         out: torch.Tensor | None = None, stage: str = "all", exact: bool = False,
         n_total: int | None = None, checked: bool = False) -> torch.Tensor:
    """Per-segment Gram stack [nseg, P, P] (fp64). ``w``: optional row weights (panel order).

    stage (paired-tile bf16 Gram): "tiles" launches only the tile kernel (slab partials),
    "reduce" only the fixed-order slab reduce into the returned buffer, "all" both. Split,
    the reduce can run on another stream than the next Gram (bench.py --stagger 2). Other
    kernels do everything at "tiles" and nothing at "reduce".

    ``exact``: world-size-invariant mode for block-aligned panels (panel.exact_block): one
    row block per chunk and the chunk partials summed as int64 limbs (ops/exact.py);
    returns the limb stack [2, nseg, P, P] (int64): all-reduce it over row shards, then
    ops.exact.from_limbs gives the same fp64 Gram at every world size (``n_total``: rows
    over all ranks, for the limb range check ``check_exact_range``; ``checked``: the
    caller already ran that check with every rank agreeing, skip it here)."""
    X = panel.data
    if exact and stage != "reduce" and not checked:
        check_exact_range(panel, n_total, w)
    if not X.is_cuda:
        if exact:
            return _gram_cpu_exact(panel, w)
        return _gram_cpu(panel, w, out) if stage != "reduce" else out
    pl = plan_for(panel, weighted=w is not None, exact=exact)
    G = pl.G if out is None else out
    Gx = pl.Gx.data_ptr() if exact else None
    s = _stream()
    if X.dtype == torch.bfloat16 and pl.tri:
        cs, bs = panel.strides()
        _native.call("ate_gram_bf16_tri", X.data_ptr(), cs, bs, panel.P, pl.blocks.data_ptr(),
                     pl.chunks.data_ptr(), pl.nchunks, pl.seg_chunk0.data_ptr(), panel.nseg,
                     pl.slab.data_ptr(), G.data_ptr(), _STAGES[stage], Gx, s)
        return pl.Gx if exact else G
    if X.dtype == torch.bfloat16 and pl.pair:
        cs, bs = panel.strides()
        x8 = getattr(panel, "bytes8", None)
        _native.call("ate_gram_bf16_pair", X.data_ptr(), cs, bs, panel.P, pl.tiles.data_ptr(),
                     pl.ntiles, pl.blocks.data_ptr(), pl.chunks.data_ptr(), pl.nchunks,
                     pl.seg_chunk0.data_ptr(), panel.nseg, pl.slab.data_ptr(), G.data_ptr(),
                     _STAGES[stage], Gx, None if x8 is None or not BYTE_COLS else x8.data_ptr(), s)
        return pl.Gx if exact else G
    if stage == "reduce":
        return pl.Gx if exact else G
    if X.dtype == torch.bfloat16:
        _native.call("ate_gram_bf16", X.data_ptr(), panel.cm_ld, panel.P, pl.T, pl.tiles.data_ptr(),
                     pl.ntiles, pl.chunks.data_ptr(), pl.nchunks, pl.seg_chunk0.data_ptr(),
                     panel.nseg, pl.slab.data_ptr(), G.data_ptr(), Gx, s)
    else:
        name = "ate_gram_f64" if X.dtype == torch.float64 else "ate_gram_f32"
        if w is not None:
            assert w.dtype == X.dtype and w.numel() == panel.ld
        _native.call(name, X.data_ptr(), panel.cm_ld, panel.P, 0 if w is None else w.data_ptr(),
                     pl.tiles.data_ptr(), pl.ntiles, pl.chunks.data_ptr(), pl.nchunks,
                     pl.seg_chunk0.data_ptr(), panel.nseg, pl.slab.data_ptr(), G.data_ptr(),
                     0 if done is None else done.data_ptr(), Gx, s)
    return pl.Gx if exact else G


def _gram_cpu(panel, w, out):
    X = panel.colmajor().double()
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


def _gram_cpu_exact(panel, w):
    """CPU twin of the exact mode: per (segment, row block) fp64 partial Grams, summed as
    int64 limbs (same block decomposition as the GPU plan)."""
    from .exact import to_limbs
    B = int(panel.exact_block)
    if B <= 0:
        raise ValueError("exact Gram needs a block-aligned panel (synthetic_panel(align=B))")
    X = panel.colmajor().double()
    out = torch.zeros((2, panel.nseg, panel.P, panel.P), dtype=torch.int64)
    for s_, (r0, r1) in enumerate(panel.seg_bounds):
        for r in range(int(r0), int(r1), B):
            e = min(int(r1), r + B)
            Xs = X[:, r:e]
            A = Xs if w is None else Xs * w[r:e].double()
            out[:, s_] += to_limbs(A @ Xs.T)
    return out


def gram_reference(panel: DevicePanel, w=None) -> torch.Tensor:
    """Plain fp64 PyTorch reference of the same op (for numerics tests)."""
    X = panel.colmajor().double().cpu()
    wv = None if w is None else w.double().cpu()
    out = []
    for (r0, r1) in panel.seg_bounds:
        Xs = X[:, r0:r1]
        A = Xs if wv is None else Xs * wv[r0:r1]
        out.append(A @ Xs.T)
    return torch.stack(out)
