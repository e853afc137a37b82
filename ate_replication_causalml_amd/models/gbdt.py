"""Histogram gradient boosting (extension nuisance learner; BASELINE config 5,
SURVEY.md K11-K14 + C04).

``fit_gbdt`` grows depth-limited trees level by level on the binned uint8 panel:
GPU (csrc/gbdt.hip) or the numpy reference (reference/gbdt.py) — same spec, same
integer histogram sums, so the same trees. With ``dist`` (row shards), each level's
node histograms are all-reduced (C04, exact int64) and every rank takes the same
split decisions; the bin edges must then be global (``global_bin_edges``).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from .. import _native
from ..reference import gbdt as ref
from . import forest as F

LOSS = {"squared": 0, "logistic": 1}


@dataclass
class GbdtModel:
    feat: object           # [T, M] int32 (-1 leaf, -2 absent)
    thr: object
    value: object          # [T, M] float64
    base: float
    loss: str
    depth: int
    edges: tuple
    backend: str

    @property
    def n_trees(self):
        return self.feat.shape[0]

    def predict(self, X, response=False):
        Xb = F.bin_matrix(np.asarray(X, dtype=np.float64), self.edges[0], self.edges[1],
                          torch.device("cuda", torch.cuda.current_device())
                          if self.backend == "gpu" else None)
        f = self.predict_binned(Xb)
        return 1.0 / (1.0 + np.exp(-f)) if (response and self.loss == "logistic") else f

    def predict_binned(self, Xb):
        n = Xb.shape[1]
        if self.backend == "gpu":
            f = torch.full((n,), self.base, dtype=torch.float64, device=Xb.device)
            M = self.feat.shape[1]
            _native.call("ate_gbdt_apply", Xb.data_ptr(), n, n, self.n_trees, M,
                         self.feat.data_ptr(), self.thr.data_ptr(), self.value.data_ptr(),
                         f.data_ptr(), torch.cuda.current_stream().cuda_stream)
            return f.cpu().numpy()
        Xn = Xb.numpy() if isinstance(Xb, torch.Tensor) else Xb
        t = ref.GbdtTrees(np.asarray(self.feat), np.asarray(self.thr), np.asarray(self.value),
                          self.base, self.loss, self.depth)
        return t.predict_binned(Xn)


def global_bin_edges(X_local, dist, rows_per_rank=20000):
    """Bin edges every rank agrees on: an evenly strided sample of each shard is
    all-gathered and binned together."""
    X_local = np.asarray(X_local, dtype=np.float64)
    if dist is None or dist.world == 1:
        return F.bin_edges(X_local)
    n = X_local.shape[0]
    take = np.linspace(0, n - 1, num=min(n, rows_per_rank)).astype(np.int64) if n else \
        np.zeros(0, dtype=np.int64)
    s = torch.zeros((rows_per_rank, X_local.shape[1]), dtype=torch.float64)
    s[:len(take)] = torch.from_numpy(X_local[take])
    cnt = torch.tensor([float(len(take))])
    counts = [int(c.item()) for c in dist.comm.all_gather(cnt)]
    parts = dist.comm.all_gather(s)
    return F.bin_edges(torch.cat([pp[:c] for pp, c in zip(parts, counts)]).numpy())


def fit_gbdt(X, y, loss="squared", n_trees=100, depth=6, lr=0.1, lam=1.0, min_child=1.0,
             min_gain=0.0, train=None, backend=None, edges=None, dist=None, seed=0) -> GbdtModel:
    """X [n, p] float, y [n]; ``train`` (bool [n]) restricts the rows the trees learn
    from (predictions still cover every row). ``seed`` is reserved for row/column
    subsampling (not used: full-data boosting is deterministic)."""
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    n, p = X.shape
    if depth < 1 or depth > 6:
        raise ValueError("depth must be in [1, 6] (<= 32 nodes per level histogram)")
    if backend is None:
        backend = "gpu" if torch.cuda.is_available() else "cpu"
    if edges is None:
        edges = global_bin_edges(X, dist)
    train = np.ones(n, dtype=bool) if train is None else np.asarray(train, dtype=bool)
    if backend != "gpu":
        Xb = F.bin_matrix(X, edges[0], edges[1], None).numpy()
        red = None
        if dist is not None and dist.world > 1:
            def red(a):
                t = torch.from_numpy(np.ascontiguousarray(a))
                return dist.sum_(t).numpy()
        tr = ref.fit(Xb, y, train, loss, n_trees, depth, lr, lam, min_child, min_gain,
                     hist_reduce=red)
        return GbdtModel(tr.feat, tr.thr, tr.value, tr.base, loss, depth, edges, "cpu")
    dev = torch.device("cuda", torch.cuda.current_device())
    s = torch.cuda.current_stream().cuda_stream
    Xb = F.bin_matrix(X, edges[0], edges[1], dev)
    yt = torch.as_tensor(y, device=dev)
    trt = torch.as_tensor(train.astype(np.uint8), device=dev)
    cnt = torch.tensor([float(y[train].sum()), float(train.sum())], dtype=torch.float64,
                       device=dev)
    if dist is not None:
        dist.sum_(cnt)
    mean = float(cnt[0] / cnt[1])
    base = mean if loss == "squared" else float(np.log(mean / (1 - mean)))
    M = 2 ** (depth + 1) - 1
    i64 = dict(dtype=torch.int64, device=dev)
    f = torch.full((n,), base, dtype=torch.float64, device=dev)
    gh = torch.empty(2 * n, **i64)
    node = torch.empty(n, dtype=torch.int32, device=dev)
    root = torch.zeros(2, **i64)
    tot = torch.zeros(2 * M, **i64)
    feat = torch.full((n_trees, M), -2, dtype=torch.int32, device=dev)
    thr = torch.zeros((n_trees, M), dtype=torch.int32, device=dev)
    value = torch.zeros((n_trees, M), dtype=torch.float64, device=dev)
    H = torch.empty(2 ** (depth - 1) * p * 512, **i64)
    mc = int(np.rint(min_child * ref.FIX))
    for t in range(n_trees):
        root.zero_()
        _native.call("ate_gbdt_grad", LOSS[loss], f.data_ptr(), yt.data_ptr(), trt.data_ptr(), n,
                     gh.data_ptr(), node.data_ptr(), root.data_ptr(), s)
        if dist is not None:
            dist.sum_(root)
        tot[:2] = root
        ft, th, vt = feat[t], thr[t], value[t]
        for d in range(depth + 1):
            nn = 2 ** d
            if d < depth:
                Hd = H[:nn * p * 512]
                Hd.zero_()
                _native.call("ate_gbdt_hist", Xb.data_ptr(), n, node.data_ptr(), gh.data_ptr(), n,
                             nn, p, Hd.data_ptr(), s)
                if dist is not None:
                    dist.sum_(Hd)
            _native.call("ate_gbdt_split", H.data_ptr(), nn, p, d, depth, lam, mc, min_gain, lr,
                         tot.data_ptr(), ft.data_ptr(), th.data_ptr(), vt.data_ptr(), s)
            if d < depth:
                _native.call("ate_gbdt_partition", Xb.data_ptr(), n, node.data_ptr(), n, d,
                             ft.data_ptr(), th.data_ptr(), s)
        _native.call("ate_gbdt_apply", Xb.data_ptr(), n, n, 1, M, ft.data_ptr(), th.data_ptr(),
                     vt.data_ptr(), f.data_ptr(), s)
    return GbdtModel(feat, thr, value, base, loss, depth, edges, "gpu")
