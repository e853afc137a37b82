"""Histogram gradient-boosted trees — the numpy reference of csrc/gbdt.hip.

Not in the R reference (SURVEY.md marks GBDT as the extension nuisance learner of
BASELINE config 5: "N=1e8 p=2000 DML with histogram-GBDT nuisance"). Spec shared by
both implementations:

* features binned to uint8 (models/forest.py::bin_edges); split "bin <= b goes left";
* per tree: gradients g and hessians h of the loss at the current prediction
  (squared: g = f - y, h = 1; logistic: s = sigmoid(f), g = s - y, h = max(s(1-s), 1e-16)),
  quantised to int64 fixed point G = rint(g * 2^28) — histogram sums are exact
  integers, so any summation order (GPU atomics, row shards + all-reduce) gives the
  same bits;
* level-wise growth to ``depth``; node totals G, H; best split of a node maximises
  GL^2/(HL+lam) + GR^2/(HR+lam) - G^2/(H+lam) over (feature, bin) subject to
  HL, HR >= min_child (in hessian units), ties -> lowest feature then lowest bin;
  split only if the gain > min_gain, else the node is a leaf;
* leaf value -lr * G / (H + lam); heap layout (children of k: 2k+1, 2k+2);
* base score: mean(y) (squared) or logit(mean(y)) (logistic) over the training rows,
  the mean taken from the EXACT sum of fix(y) (2^-28 fixed point): order-independent, so
  row-sharded fits start from the same bits at every world size.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

FIX = float(2 ** 28)


def fix(v):
    return np.rint(np.asarray(v, dtype=np.float64) * FIX).astype(np.int64)


def base_from_sums(ysum_fix: int, n: int, loss: str) -> float:
    """Base score from the exact fixed-point target sum over n training rows."""
    mean = (ysum_fix / FIX) / n
    return mean if loss == "squared" else float(np.log(mean / (1 - mean)))


def grad_hess(f, y, loss):
    if loss == "squared":
        return f - y, np.ones_like(f)
    s = 1.0 / (1.0 + np.exp(-f))
    return s - y, np.maximum(s * (1.0 - s), 1e-16)


@dataclass
class GbdtTrees:
    feat: np.ndarray     # [T, 2^(D+1)-1] int32, -1 leaf / -2 unused
    thr: np.ndarray      # [T, M] int32 bin threshold
    value: np.ndarray    # [T, M] float64 leaf values (lr applied)
    base: float
    loss: str
    depth: int

    def predict_binned(self, Xb):
        """Xb: [p, n] uint8 -> raw score."""
        n = Xb.shape[1]
        f = np.full(n, self.base)
        for t in range(self.feat.shape[0]):
            k = np.zeros(n, dtype=np.int64)
            for _ in range(self.depth + 1):
                ft = self.feat[t][k]
                inner = ft >= 0
                if not inner.any():
                    break
                b = Xb[np.where(inner, ft, 0), np.arange(n)]
                go_right = b > self.thr[t][k]
                k = np.where(inner, 2 * k + 1 + go_right, k)
            f += self.value[t][k]
        return f


def best_split(hist, G, H, lam, min_child, min_gain):
    """hist: [p, 256, 2] int64 for one node. Returns (gain, feat, bin, GL, HL) or None."""
    cg = np.cumsum(hist[:, :, 0], axis=1)
    ch = np.cumsum(hist[:, :, 1], axis=1)
    GLf, HLf = cg / FIX, ch / FIX
    Gf, Hf = G / FIX, H / FIX
    GRf, HRf = Gf - GLf, Hf - HLf
    mc = min_child
    ok = (ch >= fix(mc)) & ((H - ch) >= fix(mc))
    with np.errstate(divide="ignore", invalid="ignore"):
        gain = GLf * GLf / (HLf + lam) + GRf * GRf / (HRf + lam) - Gf * Gf / (Hf + lam)
    gain = np.where(ok, gain, -np.inf)
    flat = np.argmax(gain.reshape(-1))            # first max: lowest feature, then bin
    j, b = divmod(int(flat), gain.shape[1])
    if not np.isfinite(gain[j, b]) or not gain[j, b] > min_gain:
        return None
    return float(gain[j, b]), j, b, int(cg[j, b]), int(ch[j, b])


def fit(Xb, y, train, loss="squared", n_trees=100, depth=6, lr=0.1, lam=1.0, min_child=1.0,
        min_gain=0.0, hist_reduce=None, c04=None):
    """Xb [p, n] uint8, y [n], train [n] bool. ``hist_reduce`` (optional) sums a node
    histogram stack across row shards (the C04 all-reduce in the distributed path).
    ``c04`` (optional, with ``hist_reduce`` for the scalar sums): feature-sliced C04 --
    ``c04.scatter(hist)`` returns this rank's summed feature slice [nn, pl, 256, 2] (global
    features ``c04.joff ...``), ``c04.pick(cands)`` the best of every rank's per-node
    candidates (gain desc, feature asc, bin asc: the single-device argmax)."""
    p, n = Xb.shape
    M = 2 ** (depth + 1) - 1
    ytr = y[train]
    cnt = np.array([fix(ytr).sum(), int(train.sum())], dtype=np.int64)
    if hist_reduce is not None:
        cnt = hist_reduce(cnt)
    base = base_from_sums(int(cnt[0]), int(cnt[1]), loss)
    f = np.full(n, base)
    feat = np.full((n_trees, M), -2, dtype=np.int32)
    thr = np.zeros((n_trees, M), dtype=np.int32)
    value = np.zeros((n_trees, M))
    trees = GbdtTrees(feat, thr, value, base, loss, depth)
    rows = np.arange(n)
    for t in range(n_trees):
        g, h = grad_hess(f, y, loss)
        Gi, Hi = fix(g), fix(h)
        node = np.where(train, 0, -1)
        root = np.array([Gi[train].sum(), Hi[train].sum()], dtype=np.int64)
        if hist_reduce is not None:
            root = hist_reduce(root)
        tot = {0: (int(root[0]), int(root[1]))}
        for d in range(depth + 1):
            nn = 2 ** d
            act = node >= 0
            hist = np.zeros((nn, p, 256, 2), dtype=np.int64)
            if d < depth:
                for j in range(p):
                    idx = (node[act] * 256 + Xb[j, act]).astype(np.int64)
                    for c, w in ((0, Gi[act]), (1, Hi[act])):
                        acc = np.zeros(nn * 256, dtype=np.int64)
                        np.add.at(acc, idx, w)
                        hist[:, j, :, c] = acc.reshape(nn, 256)
                if c04 is not None:
                    hist = c04.scatter(hist)
                elif hist_reduce is not None:
                    hist = hist_reduce(hist)
            sps = [None] * nn
            for k in range(nn):
                hk = 2 ** d - 1 + k
                if d < depth and not (d > 0 and feat[t, (hk - 1) // 2] < 0):
                    sps[k] = best_split(hist[k], *tot[hk], lam, min_child, min_gain)
                    if c04 is not None and sps[k] is not None:
                        g_, j_, b_, gl_, hl_ = sps[k]
                        sps[k] = (g_, j_ + c04.joff, b_, gl_, hl_)
            if c04 is not None and d < depth:
                sps = c04.pick(sps)
            for k in range(nn):
                hk = 2 ** d - 1 + k
                if d > 0 and feat[t, (hk - 1) // 2] < 0:
                    continue                       # parent is a leaf / absent: no node
                G, H = tot[hk]
                sp = sps[k]
                if sp is None:
                    feat[t, hk] = -1
                    value[t, hk] = -lr * (G / FIX) / (H / FIX + lam)
                    continue
                _, j, b, GL, HL = sp
                feat[t, hk], thr[t, hk] = j, b
                tot[2 * hk + 1] = (GL, HL)
                tot[2 * hk + 2] = (G - GL, H - HL)
            if d == depth:
                break
            # partition: rows of split nodes move to children, rows of leaves stop
            hk = 2 ** d - 1 + np.maximum(node, 0)
            ft = feat[t, hk]
            live = act & (ft >= 0)
            b = Xb[np.where(live, ft, 0), rows]
            right = (b > thr[t, hk]).astype(np.int64)
            node = np.where(live, 2 * node + right, -1)
        f = trees_predict_one(trees, t, Xb, f)
    return trees


def trees_predict_one(trees, t, Xb, f):
    n = Xb.shape[1]
    k = np.zeros(n, dtype=np.int64)
    for _ in range(trees.depth + 1):
        ft = trees.feat[t][k]
        inner = ft >= 0
        if not inner.any():
            break
        b = Xb[np.where(inner, ft, 0), np.arange(n)]
        k = np.where(inner, 2 * k + 1 + (b > trees.thr[t][k]), k)
    return f + trees.value[t][k]
