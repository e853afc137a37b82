"""Host driver of the level-synchronous forest engine (csrc/forest_level.hip).

The GPU grows every tree of a forest together, one tree level per step; a node is decided
by many workgroups (big), one workgroup (mid) or one wave (small) according to its size,
so an 8e6-row bootstrap tree no longer lives on one CU (BASELINE config 3). Trees are the
same bits as the one-workgroup-per-tree kernel and the host twin (forest_common.hpp spec):
randomForest semantics, kinds 0 (classification) / 1 (regression), bootstrap sampling.

Per level the host reads, in one transfer, the node-class counts and the level's length
(the previous level's split count, left on the device by the children step), plus, on
levels with big nodes, their position ranges (their work items), to size the launches.
Everything else stays on the device.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from .. import _native
from ..ops.scan import exclusive_cumsum
from . import forest as F

LV_FG = 8
LV_MAXF = 64
LV_PMAX = 512


class LvHost(ctypes.Structure):
    """Mirror of csrc/forest_level.hip::LvHost."""
    P = ctypes.c_void_p
    _fields_ = [("fp", F.ForestParams), ("Xb", P), ("ycls", P), ("r1", P), ("w", P), ("idx", P),
                ("idx2", P), ("cur", P), ("dec", P), ("nl", P), ("cap", ctypes.c_int),
                ("feat", P), ("thr", P), ("left", P), ("val", P), ("depth", ctypes.c_int),
                ("fst", ctypes.c_int64), ("rst", ctypes.c_int64), ("Xc", P), ("nbin", P)]


def supported(fp: F.ForestParams) -> bool:
    return (fp.kind in (F.KIND_CLASS, F.KIND_REG) and fp.sampling == 0 and not fp.mtry_poisson
            and fp.p <= LV_PMAX and fp.mtry <= LV_MAXF and fp.ntree * fp.n < 2 ** 31 - 1)


def _env_int(name, default):
    v = os.environ.get(name)
    return int(v) if v else default


def _items(cur, sel, chunk, target, dev):
    """Work items (slot, q0, q1) cutting the nodes cur[sel] into position chunks of
    max(chunk, total / target) rows; also each slot's first item index."""
    lohi = cur.index_select(0, sel)[:, 1:3].cpu().numpy().astype(np.int64)
    lens = lohi[:, 1] - lohi[:, 0]
    ch = max(chunk, -(-int(lens.sum()) // target) // 256 * 256 + 256)
    per = -(-lens // ch)
    slot = np.repeat(np.arange(len(lens)), per)
    firsts = np.concatenate([[0], np.cumsum(per)[:-1]])
    q0 = lohi[slot, 0] + (np.arange(len(slot)) - np.repeat(firsts, per)) * ch
    q1 = np.minimum(q0 + ch, lohi[slot, 1])
    t = tuple(torch.as_tensor(a.astype(np.int32), device=dev) for a in (slot, q0, q1))
    return t, len(slot), torch.as_tensor(firsts, device=dev)


def grow(Xb: torch.Tensor, fp: F.ForestParams, yt=None, r1t=None, big=None, chunk=None,
         stream=None):
    """Grow fp.ntree trees on the device. Xb: [p][n] uint8 (cuda), yt: [n] uint8 (kind 0),
    r1t: [n] int64 fixed point (kind 1). Returns (cap, feat, thr, left, val, nnodes, inbag)."""
    dev = Xb.device
    T, n, p = fp.ntree, fp.n, fp.p
    # node classes: <= 64 rows a wave; <= t2 a workgroup + wave partition; <= t3 a
    # workgroup + chunked partition; above, many workgroups per node
    t2 = max(64, min(8192, _env_int("ATE_FOREST_LV_T2", 8192)))
    t3 = max(t2, big or _env_int("ATE_FOREST_LV_BIG", 65536))
    chunk = chunk or _env_int("ATE_FOREST_LV_CH", 4096)
    items_target = _env_int("ATE_FOREST_LV_ITEMS", 1024)
    s = (stream or torch.cuda.current_stream(dev)).cuda_stream
    i32 = dict(dtype=torch.int32, device=dev)
    cap = 2 * n + 1
    # ---- bootstrap counts, in-bag rows ascending per tree
    w = torch.zeros(T * n, **i32)
    _native.call("ate_lv_boot", ctypes.addressof(fp), w.data_ptr(), s)
    wv = w.view(T, n)
    inb = wv > 0
    inbag = inb.to(torch.uint8).reshape(-1)
    m = inb.sum(1)                                           # in-bag rows per tree
    m_h = m.cpu().numpy().astype(np.int64)
    # in-bag rows of tree t, ascending, at idx[t*n ...]: rank within the tree from a
    # lookback-free exclusive scan (ops/scan.py: this runs beside other forests' streams)
    rank = exclusive_cumsum(inb.reshape(-1).to(torch.int32)).view(T, n)
    rank = rank - rank[:, :1]
    tn = (torch.arange(T, device=dev, dtype=torch.int64) * n)[:, None]
    dest = torch.where(inb, rank.long() + tn, torch.full_like(tn, T * n))
    del rank
    idx = torch.zeros(T * n + 1, **i32)
    idx.scatter_(0, dest.reshape(-1), torch.arange(n, **i32).expand(T, n).reshape(-1))
    idx = idx[:T * n]
    idx2 = torch.zeros_like(idx)
    del dest
    # ---- outputs
    feat = torch.zeros(T * cap, **i32)
    thr = torch.zeros(T * cap, **i32)
    left = torch.zeros(T * cap, **i32)
    val = torch.zeros(T * cap, dtype=torch.float64, device=dev)
    next_id = torch.ones(T, **i32)
    # ---- level lists (capacity: every node holds >= 1 in-bag position)
    lcap = int(m_h.sum()) + T
    cur = torch.zeros((lcap, 4), **i32)
    nxt = torch.zeros((lcap, 4), **i32)
    tt = torch.arange(T, **i32)
    root = torch.stack([tt, tt * n, tt * n + m.to(torch.int32), torch.zeros_like(tt)], 1)
    keep = np.flatnonzero(m_h > 0)
    if len(keep) < T:
        root = root.index_select(0, torch.as_tensor(keep, device=dev))
    ncur = int(root.shape[0])
    cur[:ncur] = root
    dec = torch.zeros((lcap, 4), **i32)
    nl = torch.zeros(lcap, **i32)
    brank = torch.zeros(T, **i32)
    counts = torch.zeros(5, **i32)
    nsplit = None            # device [1]: split count of the previous level (None: root level)
    nf_max = min(fp.mtry, p)
    ngroups = -(-nf_max // LV_FG)
    hist = None
    # Row-major bins for the growth: a node's rows are scattered over the n positions, so
    # each (row, feature) gather of a column-major [p][n] matrix touches its own cache
    # line; in a row-major [n][p] copy a row's drawn features share that row's few lines
    # (22 of 500 bytes: ~4 lines instead of 22). One transpose (n x p bytes) per forest.
    if os.environ.get("ATE_FOREST_LV_LAYOUT", "row") == "row":
        ldr = -(-p // 16) * 16
        Xg = torch.empty((n, ldr), dtype=torch.uint8, device=dev)
        _native.call("ate_lv_transpose", Xb.data_ptr(), p, n, Xg.data_ptr(), ldr, s)
        fst, rst = 1, ldr
    else:
        Xg, fst, rst = Xb, n, 1
    # bins per feature (max bin + 1 over the training rows): few-bin features spread their
    # LDS histograms over the 256 slots (csrc/forest_level.hip lv_spread)
    nbin = (Xb.amax(dim=1).to(torch.int32) + 1).to(torch.int16).contiguous()
    h = LvHost(fp=fp, Xb=Xg.data_ptr(), Xc=Xb.data_ptr(), nbin=nbin.data_ptr(),
               ycls=yt.data_ptr() if yt is not None else None,
               r1=r1t.data_ptr() if r1t is not None else None, w=w.data_ptr(), cap=cap,
               feat=feat.data_ptr(), thr=thr.data_ptr(), left=left.data_ptr(),
               val=val.data_ptr(), fst=fst, rst=rst)
    prof = os.environ.get("ATE_FOREST_LV_PROF") == "1"
    if prof:
        import time
        tp = {"classify": 0.0, "decide": 0.0, "partition": 0.0, "children": 0.0}
        lv_rows = []
        torch.cuda.current_stream(dev).synchronize()
        t_all = time.perf_counter()

    def tick(name, t0):
        if not prof:
            return None
        torch.cuda.current_stream(dev).synchronize()
        t1 = time.perf_counter()
        if name:
            tp[name] += t1 - t0
        return t1
    depth = 0
    ncur_ub = ncur           # upper bound of the level length (exact at the root)
    while ncur_ub > 0:
        t0 = tick(None, None)
        h.idx, h.idx2 = idx.data_ptr(), idx2.data_ptr()
        h.cur, h.dec, h.nl = cur.data_ptr(), dec.data_ptr(), nl.data_ptr()
        h.depth = depth
        lists = torch.empty(4 * ncur_ub, **i32)
        counts.zero_()
        _native.call("ate_lv_classify", cur.data_ptr(), ncur_ub,
                     nsplit.data_ptr() if nsplit is not None else None, t2, t3,
                     lists.data_ptr(), counts.data_ptr(), s)
        nsmall, nmid, nmid2, nbig, ncur = (int(v) for v in counts.cpu())   # the level's sync
        if ncur == 0:
            break
        t0 = tick("classify", t0) if prof else None
        L = [lists[k * ncur_ub:k * ncur_ub + c] for k, c in enumerate((nsmall, nmid, nmid2, nbig))]
        P = lambda t: t.data_ptr() if t is not None else None
        items, nitems, drawn, nfo = (None, None, None), 0, None, None
        if nbig:
            items, nitems, _ = _items(cur, L[3].long(), chunk, items_target, dev)
            drawn = torch.empty(nbig * LV_MAXF, dtype=torch.int16, device=dev)
            nfo = torch.empty(nbig, **i32)
            need = nbig * nf_max * 2 * F.MAX_BINS
            if hist is None or hist.numel() < need:
                hist = torch.empty(need, dtype=torch.int64, device=dev)
            hist[:need].zero_()
        _native.call("ate_lv_decide", ctypes.addressof(h), P(L[0]), nsmall, P(L[1]), nmid,
                     P(L[2]), nmid2, P(L[3]), nbig, P(drawn), P(nfo), P(items[0]), P(items[1]),
                     P(items[2]), nitems, ngroups, P(hist), nf_max, s)
        if prof:
            td = tick("decide", t0)
            lv_rows.append((depth, ncur, nsmall, nmid, nmid2, nbig, td - t0))
            t0 = td
        # partition: small + mid by waves, mid-large + big by position chunks
        plist = torch.cat([L[2], L[3]]) if nmid2 + nbig else None
        pitems, npit, firsts = (None, None, None), 0, None
        if plist is not None:
            pitems, npit, firsts = _items(cur, plist.long(), chunk, 4 * items_target, dev)
        icnt = torch.empty(max(npit, 1), **i32)
        _native.call("ate_lv_partition", ctypes.addressof(h), P(L[0]), nsmall, P(L[1]), nmid,
                     P(plist), P(pitems[0]), P(pitems[1]), P(pitems[2]), npit, icnt.data_ptr(), s)
        if npit:
            ic = icnt[:npit].long()
            slot_t = pitems[0].long()
            csum = exclusive_cumsum(ic)
            ipre = (csum - csum.index_select(0, firsts).index_select(0, slot_t)).to(torch.int32)
            nlb = torch.zeros(plist.numel(), dtype=torch.int64, device=dev).index_add_(0, slot_t, ic)
            nlb32 = nlb.to(torch.int32)
            nl.index_copy_(0, plist.long(), nlb32)
            _native.call("ate_lv_scatter", ctypes.addressof(h), P(plist), P(pitems[0]),
                         P(pitems[1]), P(pitems[2]), npit, ipre.data_ptr(), nlb32.data_ptr(), s)
        t0 = tick("partition", t0) if prof else None
        flags = dec[:ncur, 0]
        excl, nsplit = exclusive_cumsum(flags.contiguous(), total=True)   # stays on device
        _native.call("ate_lv_children", ctypes.addressof(h), ncur, excl.data_ptr(),
                     brank.data_ptr(), next_id.data_ptr(), nxt.data_ptr(), s)
        if prof:
            tick("children", t0)
        cur, nxt = nxt, cur
        idx, idx2 = idx2, idx
        ncur_ub = 2 * ncur   # each node has at most two children
        depth += 1
    if prof:
        import sys
        tot = time.perf_counter() - t_all
        top = sorted(lv_rows, key=lambda r: -r[-1])[:6]
        print(f"[forest_level] T={T} n={n} levels={depth} {tot:.3f}s "
              + " ".join(f"{k}={v:.3f}" for k, v in tp.items())
              + " slowest decide levels (depth,ncur,small,mid,mid2,big,s): "
              + "; ".join(f"{r[0]},{r[1]},{r[2]},{r[3]},{r[4]},{r[5]},{r[6]:.3f}" for r in top),
              file=sys.stderr, flush=True)
    return cap, feat, thr, left, val, next_id, inbag
