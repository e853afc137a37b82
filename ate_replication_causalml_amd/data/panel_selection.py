"""Selection-bias transform at panel scale (K04, SURVEY.md §2.8 last bullet).

The tutorial's estimators all run on ``df_mod``: the rows left after dropping the FIRST
round(0.85 k) treated "likely voters" and control "unlikely voters" in row order
(``ate_replication.Rmd:99-121``, quirks Q17/Q18; host version data/selection.py). For the
scaled configs the transform is applied to GENERATED rows (global row id g, a pure Philox
function of (seed, g)) before any panel row is written:

1. **Candidate counts** (``csrc/dgp.hip`` sel_gen_count): per block of ``SEL_BR`` generated
   rows, the treated and control candidates -- nine Philox draws per row, no panel. Each
   rank counts its contiguous share of the blocks; one all-reduce of the int64 count vector
   gives every rank the counts of all blocks (the cross-rank prefix of "first k in global
   row order").
2. **n_gen and thresholds** (host, exact integers): the kept count of the first n generated
   rows, kept(n) = n - round(pt ct(n)) - round(pc cc(n)), steps by 0 or 1, so the smallest n
   with kept(n) = N exists; it is found at block granularity from the counts, then inside
   one block from its flags. The transform of the first n_gen rows keeps exactly N rows;
   thr_t = round(pt ct(n_gen)), thr_c = round(pc cc(n_gen)) (R's round: half to even).
3. **Kept ids** (sel_gen_mark): a rank's panel holds kept-row slices (kept rank q -> fold
   q K // N, rank r the r-th slice of every fold: device_dgp.fold_slices); the blocks that
   cover them are re-flagged, candidates ranked from the block prefix counts, and the
   generated ids of the kept rows written in kept-rank order. The panel is then filled
   from that id list (ate_dgp_fill).

Every rank derives the same n_gen / thresholds / kept set from the same integers, so the
union of the shards is the same data set at every world size. On a CPU panel the flags
come from the host (dgp.selection_flags), on the GPU from the device kernels: both compute
the draws the rule reads in fp64 with the same formulas (csrc/dgp.hip core_draws, no FMA
contraction), so a CPU panel and a GPU panel of the same (N, seed) keep the same rows
(tests/test_gpu_panel_selection.py; a flag could differ only for a draw within an ulp of a
threshold, where the two log / cos implementations may round differently).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from .. import _native
from .dgp import DgpParams, selection_flags

SEL_BR = 16384            # generated rows per selection block (csrc/dgp.hip SEL_BR)
KEEP_FRACTION_GUESS = 0.16
MAX_SEL_BLOCKS = 1 << 20   # 1.7e10 generated rows: far past any config (config 5: 4.2e8)


def r_round(x: float) -> int:
    """R's round(): IEC 60559 half to even."""
    return int(np.round(x))


@dataclass
class PanelSelection:
    n_keep: int
    n_gen: int             # generated rows the transform ran over
    thr_t: int             # treated candidates dropped (the first thr_t in row order)
    thr_c: int
    cand_t: int            # treated / control candidates among the n_gen rows
    cand_c: int
    blk_ct: np.ndarray     # per block (of the first ceil(n_gen / SEL_BR)): treated candidates
    blk_cc: np.ndarray
    blk_kept: np.ndarray   # kept rows per block
    kp: np.ndarray         # exclusive prefix of blk_kept
    seed: int
    params: DgpParams
    compat: str

    @property
    def nblk(self):
        return len(self.blk_kept)

    @property
    def last(self):
        return 3 if self.compat == "reference" else 4


def _allreduce_counts(t: torch.Tensor, comm):
    if comm is None or comm.world_size == 1:
        return t
    if getattr(comm, "capturable", False) or not t.is_cuda:
        comm.all_reduce_(t)
        return t
    h = t.cpu()                   # gloo with device tensors: host-staged
    comm.all_reduce_(h)
    return t.copy_(h)


class _Flags:
    """Flag source: the device kernels (cuda) or the float64 host twin (cpu)."""

    def __init__(self, seed, params: DgpParams, compat, device):
        self.seed, self.params, self.compat = int(seed), params, compat
        self.dev = torch.device(device)
        self.gpu = self.dev.type == "cuda"
        self.last = 3 if compat == "reference" else 4
        if self.gpu:
            if _native.hip().ate_sel_block_rows() != SEL_BR:
                raise RuntimeError("csrc/dgp.hip SEL_BR differs from data/panel_selection.py")
            self.pblk = np.ascontiguousarray(params.device_block())

    def _stream(self):
        return torch.cuda.current_stream(self.dev).cuda_stream

    def counts(self, b0: int, nblk: int, n_lim: int) -> torch.Tensor:
        """int64 [nblk, 2] candidate counts of blocks [b0, b0 + nblk)."""
        if self.gpu:
            out = torch.zeros((max(nblk, 0), 2), dtype=torch.int64, device=self.dev)
            _native.call("ate_sel_gen_count", self.seed, self.pblk.ctypes.data, self.last,
                         b0, nblk, n_lim, out.data_ptr(), self._stream())
            return out
        out = torch.zeros((max(nblk, 0), 2), dtype=torch.int64)
        for i in range(nblk):
            g0 = (b0 + i) * SEL_BR
            g1 = min(g0 + SEL_BR, n_lim)
            if g1 <= g0:
                continue
            f = self.flags(g0, g1 - g0)
            out[i, 0] = int((f == 1).sum())
            out[i, 1] = int((f == 2).sum())
        return out

    def flags(self, g0: int, count: int) -> np.ndarray:
        if self.gpu:
            f = torch.empty(count, dtype=torch.uint8, device=self.dev)
            _native.call("ate_sel_gen_flags", self.seed, self.pblk.ctypes.data, self.last, g0,
                         count, f.data_ptr(), self._stream())
            return f.cpu().numpy()
        return selection_flags(self.seed, np.arange(g0, g0 + count, dtype=np.uint64),
                               self.params, self.compat)


def plan_selection(n_keep: int, seed: int, params: DgpParams, comm=None, device="cpu",
                   pt: float = 0.85, pc: float = 0.85, compat: str = "reference") -> PanelSelection:
    """Find n_gen (the generated rows whose transform keeps exactly ``n_keep``) and the
    per-block counts. Blocks are counted sharded over ``comm`` (without one, a rank counts
    every block itself: the same integers)."""
    if not (0 < pt <= 1 and 0 < pc <= 1):
        raise ValueError("pt, pc must be in (0, 1]")
    if int(n_keep) < 1:
        raise ValueError(f"n_keep must be >= 1, got {n_keep}")
    fl = _Flags(seed, params, compat, device)
    r, w = (comm.rank, comm.world_size) if comm is not None else (0, 1)
    ct = np.zeros(0, np.int64)
    cc = np.zeros(0, np.int64)
    guess = KEEP_FRACTION_GUESS
    while True:
        # blocks to have counted: enough for n_keep at the keep fraction seen so far (+3 %)
        want = int(np.ceil(n_keep / guess * 1.03 / SEL_BR)) + 1
        if want > MAX_SEL_BLOCKS:
            # every rank sees the same counts, so every rank raises here together
            raise ValueError(f"the selection keeps too few rows: {n_keep} kept rows would "
                             f"need more than {MAX_SEL_BLOCKS * SEL_BR} generated rows")
        have = len(ct)
        if want > have:
            n_new = want - have
            a = have + r * n_new // w
            b = have + (r + 1) * n_new // w
            part = torch.zeros((n_new, 2), dtype=torch.int64, device=fl.dev)
            if b > a:
                part[a - have:b - have] = fl.counts(a, b - a, 1 << 62)
            part = _allreduce_counts(part, comm)
            ph = part.cpu().numpy()
            ct = np.concatenate([ct, ph[:, 0]])
            cc = np.concatenate([cc, ph[:, 1]])
        CT = np.concatenate([[0], np.cumsum(ct)])
        CC = np.concatenate([[0], np.cumsum(cc)])
        nb = np.arange(len(CT), dtype=np.int64) * SEL_BR
        kept = np.array([int(nb[i]) - r_round(pt * int(CT[i])) - r_round(pc * int(CC[i]))
                         for i in range(len(CT))], dtype=np.int64)
        hit = np.flatnonzero(kept >= n_keep)
        if len(hit):
            break
        guess = max(1e-3, kept[-1] / max(1, nb[-1]) * 0.97)
    b = int(hit[0])                     # kept(b SEL_BR) >= n_keep > kept((b-1) SEL_BR)
    g0 = (b - 1) * SEL_BR
    f = fl.flags(g0, SEL_BR)
    ct_in = int(CT[b - 1]) + np.cumsum(f == 1)
    cc_in = int(CC[b - 1]) + np.cumsum(f == 2)
    n_in = g0 + np.arange(1, SEL_BR + 1)
    kept_in = np.array([int(n_in[i]) - r_round(pt * int(ct_in[i])) - r_round(pc * int(cc_in[i]))
                        for i in range(SEL_BR)])
    i = int(np.flatnonzero(kept_in >= n_keep)[0])
    n_gen = int(n_in[i])
    kt, kc = int(ct_in[i]), int(cc_in[i])
    if kept_in[i] != n_keep:
        raise AssertionError("selection kept count skipped a value")
    thr_t, thr_c = r_round(pt * kt), r_round(pc * kc)
    nblk = -(-n_gen // SEL_BR)
    bct = ct[:nblk].copy()
    bcc = cc[:nblk].copy()
    bct[-1] = kt - int(CT[nblk - 1])    # the last block only up to n_gen
    bcc[-1] = kc - int(CC[nblk - 1])
    CTx = np.concatenate([[0], np.cumsum(bct)[:-1]])
    CCx = np.concatenate([[0], np.cumsum(bcc)[:-1]])
    rows = np.minimum(SEL_BR, n_gen - np.arange(nblk, dtype=np.int64) * SEL_BR)
    dt = np.clip(thr_t - CTx, 0, bct)
    dc = np.clip(thr_c - CCx, 0, bcc)
    bk = rows - dt - dc
    kp = np.concatenate([[0], np.cumsum(bk)[:-1]])
    if int(bk.sum()) != n_keep:
        raise AssertionError("selection block kept counts do not add up")
    return PanelSelection(n_keep, n_gen, thr_t, thr_c, kt, kc, bct, bcc, bk, kp, int(seed),
                          params, compat)


def kept_gids(sel: PanelSelection, slices, device="cpu") -> torch.Tensor:
    """Generated ids of the kept rows in kept-rank slices ``[(start, count), ...]`` (sorted,
    disjoint), concatenated in slice order (int64 on ``device``)."""
    dev = torch.device(device)
    total = int(sum(c for _, c in slices))
    sl = []
    off = 0
    for a, c in slices:
        sl.append((int(a), int(a) + int(c), off))
        off += int(c)
    ends = sel.kp + sel.blk_kept
    need = set()
    for a, e, _ in sl:
        if e <= a:
            continue
        b0 = int(np.searchsorted(ends, a, side="right"))     # first block with end > a
        b1 = int(np.searchsorted(sel.kp, e, side="left"))    # blocks with start < e
        need.update(range(b0, b1))
    need = sorted(need)
    if dev.type == "cuda":
        out = torch.full((max(total, 1),), -1, dtype=torch.int64, device=dev)
        if need:
            CTx = np.concatenate([[0], np.cumsum(sel.blk_ct)[:-1]])
            CCx = np.concatenate([[0], np.cumsum(sel.blk_cc)[:-1]])
            tab = np.zeros((len(need), 6), dtype=np.int64)
            for j, b in enumerate(need):
                tab[j] = (b * SEL_BR, min((b + 1) * SEL_BR, sel.n_gen), CTx[b], CCx[b], sel.kp[b], 0)
            blk = torch.from_numpy(tab.reshape(-1)).to(dev)
            slt = torch.from_numpy(np.asarray(sl, dtype=np.int64).reshape(-1)).to(dev)
            pblk = np.ascontiguousarray(sel.params.device_block())
            _native.call("ate_sel_gen_mark", sel.seed, pblk.ctypes.data, sel.last, blk.data_ptr(),
                         len(need), sel.thr_t, sel.thr_c, slt.data_ptr(), len(sl), out.data_ptr(),
                         total, torch.cuda.current_stream(dev).cuda_stream)
            torch.cuda.current_stream(dev).synchronize()    # pblk / tables are host-owned
        out = out[:total]
        if total and bool((out < 0).any()):
            raise AssertionError("selection left a kept-row slot unfilled")
        return out
    # host twin: same integers, flags from dgp.selection_flags
    out = np.full(total, -1, dtype=np.int64)
    CTx = np.concatenate([[0], np.cumsum(sel.blk_ct)[:-1]])
    CCx = np.concatenate([[0], np.cumsum(sel.blk_cc)[:-1]])
    for b in need:
        g0, g1 = b * SEL_BR, min((b + 1) * SEL_BR, sel.n_gen)
        g = np.arange(g0, g1, dtype=np.int64)
        f = selection_flags(sel.seed, g.astype(np.uint64), sel.params, sel.compat)
        rt = CTx[b] + np.cumsum(f == 1) - 1
        rc = CCx[b] + np.cumsum(f == 2) - 1
        drop = ((f == 1) & (rt < sel.thr_t)) | ((f == 2) & (rc < sel.thr_c))
        k = ~drop
        q = sel.kp[b] + np.cumsum(k) - 1
        for a, e, o in sl:
            m = k & (q >= a) & (q < e)
            out[o + q[m] - a] = g[m]
    if total and (out < 0).any():
        raise AssertionError("selection left a kept-row slot unfilled")
    return torch.from_numpy(out)


def selected_rows(n_keep: int, seed: int, p_extra: int = 0, compat: str = "reference",
                  device="cpu"):
    """The tutorial's df_mod at any size as host arrays (dgp.TutorialData): the calibrated
    model's generated rows, selected by the transform over generated-row order (flags on
    ``device``: the GPU's float32 draws or the host's float64 twin), then the kept rows'
    columns drawn on the host (population-standardised continuous covariates, as the
    panels; configs 3 / 4 on host-resident data: tools/cfg4.py)."""
    from . import dgp as D
    sel = plan_selection(n_keep, seed, D.TUTORIAL, device=device, compat=compat)
    g = kept_gids(sel, [(0, n_keep)], device=device).cpu().numpy()
    cts, binc, extra, W, Y, tau_i = D.raw_columns(n_keep, seed, p_extra, params=D.TUTORIAL,
                                                  idx=g)
    names = list(D.COVARIATES) + [f"x_extra{j}" for j in range(p_extra)]
    X = np.column_stack([cts, binc, extra]) if p_extra else np.column_stack([cts, binc])
    return D.TutorialData(X=X, W=W, Y=Y, names=names, tau_true=float(tau_i.mean())), sel
