"""Reference (T-ref) forests, written independently of the engines in numpy: trees grown one
node at a time from the forest specification (csrc/forest_common.hpp header) -- the
randomForest / grf semantics of SURVEY.md N5/N6 (``ate_functions.R:169-174,340-349``,
``ate_replication.Rmd:250-265``) on uint8 quantile bins or, in exact-split mode, uint16
ranks of every feature's distinct values.

It shares nothing with csrc/cpu/forest_cpu.cpp or the gfx950 kernels but the spec: the
Philox streams (parallel/rng.py), the 2^-32 fixed-point statistics, the criteria and their
tie-breaks. Tests grow small forests here and with both engines and require the same
trees (feature, threshold bin, child index, leaf value) and the same honest estimation
sums, node for node. Slow by design (a Python loop per node and candidate feature): a
parity oracle for n of a few hundred rows.

Spec, per tree ``tg`` (global tree index, the RNG stream):
  rows      sampling 0: bootstrap counts w = multinomial(n; 1/n) from Philox(P_RF_BOOT, tg);
            sampling 1: grf half-samples by Algorithm S (P_SUBSAMPLE): little bag H of
            floor(n/2) rows per group (stream tg // group), the tree's subsample of H (or of
            all rows when group == 1; stream 0x10000 + tg), honesty's random half J1
            (stream 0x20000 + tg) grows the tree (w = 1), the rest J2 fills ``est``;
  nodes     breadth first; children of the k-th split of the tree get ids 2k+1, 2k+2;
  features  a partial Fisher-Yates shuffle of 0..p-1 with Philox(P_RF_MTRY, tg,
            node * 4096 + k), the first nf slots tried (grf: nf ~ Poisson(mtry), one
            uniform at index node * 4096 + 4094, inverse CDF, clamped to [1, p]);
  splits    every boundary between two consecutive distinct bins present in the node
            (left = bins <= the lower one) of every tried feature, in (slot, bin) order,
            strict improvement: the first maximum wins (exact-split mode: bins are value
            ranks; randomForest places the threshold at the values' midpoint, grf at the
            lower value); each child needs
            minc = max(ceil(alpha * n_node), 1) rows (causal: grf's stabilize.splits rule,
            minc rows with W~ below the node mean AND minc rows with W~ >= it in each
            child); split only if best > parent + 1e-12 max(1,
            |parent|) and the node has more than ``min_node`` rows (not pure, kind 0;
            Var(W~) > 0, kind 2); at most 64 levels;
  leaves    kind 0: majority vote of the weighted class counts, ties by a Philox coin at
            node * 4096 + 4095; kind 1: weighted mean response; kind 2: 0 (grf predicts from
            the J2 statistics).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from ..parallel import rng

P_RF_BOOT, P_RF_MTRY, P_SUBSAMPLE = 3, 4, 6
NBINS = 256
MAX_DEPTH = 64
FIX = 4294967296.0


def to_fix(v: float) -> int:
    s = float(v) * FIX
    return int(s + 0.5) if s >= 0 else int(s - 0.5)      # round half away from zero


def from_fix(v: int) -> float:
    return float(v) / FIX


def _u32(seed, purpose, stream, index):
    return int(rng.random_u32(seed, purpose, np.uint32(stream), np.uint64(index))[0])


def _below(seed, purpose, stream, index, n):
    return (_u32(seed, purpose, stream, index) * n) >> 32


def _algorithm_s(seed, pop, k, stream):
    """Knuth's selection sampling of k of the (ordered) population, one Philox uniform per
    visited element: element i joins iff u24 * (N - i) < (k - taken) * 2^24."""
    N = len(pop)
    u24 = (rng.random_u32(seed, P_SUBSAMPLE, np.uint32(stream),
                          np.arange(N, dtype=np.uint64))[:, 0] >> np.uint32(8)).astype(np.int64)
    out = []
    for i in range(N):
        if len(out) >= k:
            break
        if int(u24[i]) * (N - i) < (k - len(out)) << 24:
            out.append(pop[i])
    return out


@dataclass
class Params:
    kind: int                 # 0 classification, 1 regression, 2 causal
    sampling: int = 0         # 0 bootstrap, 1 grf half-samples
    mtry: int = 1
    min_node: int = 1
    honesty: bool = False
    group: int = 1
    mtry_poisson: bool = False
    alpha: float = 0.0
    sample_fraction: float = 0.5
    seed: int = 1


def _tree_rows(P: Params, n: int, tg: int):
    """(weights w [n], in-bag flags [n], estimation rows) of tree tg."""
    if P.sampling == 0:
        idx = rng.randint(P.seed, P_RF_BOOT, np.uint32(tg), np.arange(n, dtype=np.uint64), n)
        w = np.bincount(idx, minlength=n).astype(np.int64)
        return w, (w > 0).astype(np.uint8), []
    inb = np.zeros(n, dtype=np.uint8)
    if P.group > 1:
        H = _algorithm_s(P.seed, list(range(n)), n // 2, tg // P.group)
        inb[H] = 1
        f = min(P.sample_fraction * P.group, 1.0)
        S = H if f >= 1.0 else _algorithm_s(P.seed, H, int(math.floor(len(H) * f)),
                                            0x10000 + tg)
    else:
        S = _algorithm_s(P.seed, list(range(n)), int(math.floor(n * P.sample_fraction)),
                         0x10000 + tg)
        inb[S] = 1
    J1 = S
    est = list(S)
    if P.honesty:
        J1 = _algorithm_s(P.seed, S, len(S) // 2, 0x20000 + tg)
        j1 = set(J1)
        est = [i for i in S if i not in j1]
    w = np.zeros(n, dtype=np.int64)
    w[J1] = 1
    return w, inb, est


def _num_features(P: Params, p: int, tg: int, v: int) -> int:
    if not P.mtry_poisson:
        return min(P.mtry, p)
    u = (_u32(P.seed, P_RF_MTRY, tg, v * 4096 + 4094) >> 8) * (1.0 / 16777216.0)
    lam = float(P.mtry)
    pmf = math.exp(-lam)
    cdf, k = pmf, 0
    while u > cdf and k < 4 * P.mtry + 64:
        k += 1
        pmf = pmf * lam / k
        cdf += pmf
    return max(1, min(k, p))


def _tried_features(P: Params, p: int, tg: int, v: int, nf: int):
    perm = list(range(p))
    for k in range(nf):
        r = _below(P.seed, P_RF_MTRY, tg, v * 4096 + k, p - k)
        perm[k], perm[k + r] = perm[k + r], perm[k]
    return perm[:nf]


def grow_tree(Xb, P: Params, tg: int, y=None, r1=None, r2=None, exact=None):
    """One tree. Xb [p, n] uint8 bins, or with ``exact`` (models/forest.ExactBins: sorted
    distinct values per feature) uint16 value ranks; y 0/1 (kind 0); r1 (and r2, kind 2)
    2^-32 fixed-point int64 responses (kind 1: Y; kind 2: W~, Y~). Returns dict of node
    arrays (feat, thr, left, val), the in-bag flags and, for sampling 1, est [nodes, 5]."""
    p, n = Xb.shape
    w, inb, est_rows = _tree_rows(P, n, tg)
    feat, thr, left, val = [], [], [], []

    def node_slot(v):
        while len(feat) <= v:
            feat.append(-1)
            thr.append(-1)
            left.append(-1)
            val.append(0.0)

    rows0 = [i for i in range(n) if w[i] > 0]
    level = [(0, rows0)]
    next_id = 1
    depth = 0
    while level:
        nxt = []
        for v, rows in level:
            node_slot(v)
            rows_a = np.asarray(rows, dtype=np.int64)
            wr = w[rows_a]
            nw = int(wr.sum())
            terminal = nw <= P.min_node or depth >= MAX_DEPTH - 1
            n1 = s1 = 0
            if P.kind == 0:
                n1 = int((wr * y[rows_a]).sum())
                terminal = terminal or n1 == 0 or n1 == nw
            elif P.kind == 1:
                s1 = int((wr * r1[rows_a]).sum())
            else:
                sw = sum(int(r1[i]) for i in rows)
                sy = sum(int(r2[i]) for i in rows)
                sww = sum(to_fix(from_fix(r1[i]) * from_fix(r1[i])) for i in rows)
                swy = sum(to_fix(from_fix(r1[i]) * from_fix(r2[i])) for i in rows)
                dn = float(nw)
                wbar, ybar = from_fix(sw) / dn, from_fix(sy) / dn
                cww = from_fix(sww) / dn - wbar * wbar
                cwy = from_fix(swy) / dn - wbar * ybar
                tau = cwy / cww if cww > 0.0 else 0.0
                terminal = terminal or not cww > 0.0
            best_f = best_b = -1
            if not terminal:
                dn = float(nw)
                if P.kind == 0:
                    a, b = float(nw - n1), float(n1)
                    parent = (a * a + b * b) / dn
                    stat = None
                else:
                    if P.kind == 1:
                        stat = {i: int(w[i]) * int(r1[i]) for i in rows}
                    else:
                        def rho(i):
                            dw = from_fix(r1[i]) - wbar
                            r = dw * ((from_fix(r2[i]) - ybar) - tau * dw)
                            return to_fix(r / cww if cww > 0.0 else 0.0)
                        stat = {i: rho(i) for i in rows}
                    stot = sum(stat.values())
                    sd = from_fix(stot)
                    parent = sd * sd / dn
                minc = 1 if P.alpha <= 0.0 else max(1, int(math.ceil(P.alpha * dn)))
                treated = {i: P.kind == 2 and from_fix(r1[i]) >= wbar for i in rows}
                ntreat = sum(treated.values())
                best = -math.inf
                for f in _tried_features(P, p, tg, v, _num_features(P, p, tg, v)):
                    # the node's rows in ascending bin order; a candidate split sits between
                    # every two consecutive DISTINCT bins present in the node (an empty bin
                    # boundary repeats the previous partition, never strictly better)
                    srt = sorted(rows, key=lambda i: (int(Xb[f, i]), i))
                    cl = c1 = cs = ct = 0
                    for q in range(len(srt) - 1):
                        i = srt[q]
                        cl += int(w[i])
                        if P.kind == 0:
                            c1 += int(w[i]) * int(y[i])
                        else:
                            cs += stat[i]
                            ct += int(treated[i])
                        b, bn = int(Xb[f, i]), int(Xb[f, srt[q + 1]])
                        if b == bn:
                            continue
                        nl, nr = cl, nw - cl
                        if nl < minc or nr < minc:
                            continue
                        if P.kind == 0:
                            l0, l1 = float(cl - c1), float(c1)
                            q0, q1 = float(nw - n1 - (cl - c1)), float(n1 - c1)
                            crit = (l0 * l0 + l1 * l1) / (l0 + l1) + (q0 * q0 + q1 * q1) / (q0 + q1)
                        else:
                            if P.kind == 2:
                                tr = ntreat - ct
                                if ct < minc or nl - ct < minc or tr < minc or nr - tr < minc:
                                    continue
                            sl, sr = from_fix(cs), from_fix(stot - cs)
                            crit = (sl * sl) / float(nl) + (sr * sr) / float(nr)
                        if crit > best:
                            best, best_f, best_b, best_bn = crit, f, b, bn
                if not (best_f >= 0 and best > parent + 1e-12 * max(1.0, abs(parent))):
                    best_f = -1
            if best_f < 0:
                if P.kind == 0:
                    if 2 * n1 > nw:
                        vote = 1
                    elif 2 * n1 < nw:
                        vote = 0
                    else:
                        vote = _u32(P.seed, P_RF_MTRY, tg, v * 4096 + 4095) & 1
                    val[v] = float(vote)
                elif P.kind == 1:
                    val[v] = from_fix(s1) / float(nw)
                continue
            if exact is not None and P.sampling == 0:
                # randomForest: the midpoint of the two values, as the largest value rank
                # <= it, kept inside [blo, bhi - 1]
                vals = exact.vals[best_f, :exact.nval[best_f]]
                mid = (vals[best_b] + vals[best_bn]) / 2.0
                best_b = min(max(int(np.searchsorted(vals, mid, side="right")) - 1, best_b),
                             best_bn - 1)
            lrows = [i for i in rows if Xb[best_f, i] <= best_b]
            rrows = [i for i in rows if Xb[best_f, i] > best_b]
            feat[v], thr[v], left[v] = best_f, best_b, next_id
            nxt.append((next_id, lrows))
            nxt.append((next_id + 1, rrows))
            next_id += 2
        level = nxt
        depth += 1
    node_slot(next_id - 1)
    out = dict(feat=np.array(feat[:next_id], dtype=np.int32),
               thr=np.array(thr[:next_id], dtype=np.int32),
               left=np.array(left[:next_id], dtype=np.int32),
               val=np.array(val[:next_id]), inbag=inb, nnodes=next_id)
    if P.sampling == 1:
        est = np.zeros((next_id, 5), dtype=np.int64)
        for i in est_rows:
            v = 0
            while True:
                est[v, 0] += 1
                est[v, 1] += int(r1[i])
                if P.kind == 2:
                    est[v, 2] += int(r2[i])
                    est[v, 3] += to_fix(from_fix(r1[i]) * from_fix(r1[i]))
                    est[v, 4] += to_fix(from_fix(r1[i]) * from_fix(r2[i]))
                if out["feat"][v] < 0:
                    break
                v = int(out["left"][v]) + (0 if Xb[out["feat"][v], i] <= out["thr"][v] else 1)
        out["est"] = est
    return out


def grow_forest(Xb, P: Params, ntree: int, y=None, r1=None, r2=None, t0: int = 0, exact=None):
    """Trees t0 .. t0 + ntree - 1 (``grow_tree`` each)."""
    Xb = np.asarray(Xb)
    y = None if y is None else np.asarray(y).astype(np.int64)
    r1 = None if r1 is None else np.asarray(r1, dtype=np.int64)
    r2 = None if r2 is None else np.asarray(r2, dtype=np.int64)
    return [grow_tree(Xb, P, t0 + t, y, r1, r2, exact) for t in range(ntree)]


def predict_mean(trees, Xb, oob=False):
    """kind 0 / 1 with bootstrap sampling: the mean over (out-of-bag) trees of the leaf
    value each row falls in -- randomForest's vote share / regression prediction."""
    Xb = np.asarray(Xb)
    n = Xb.shape[1]
    tot, cnt = np.zeros(n), np.zeros(n)
    for tr in trees:
        for i in range(n):
            if oob and tr["inbag"][i]:
                continue
            v = 0
            while tr["feat"][v] >= 0:
                v = int(tr["left"][v]) + (0 if Xb[tr["feat"][v], i] <= tr["thr"][v] else 1)
            tot[i] += tr["val"][v]
            cnt[i] += 1
    with np.errstate(invalid="ignore"):
        return tot / cnt
