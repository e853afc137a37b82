"""Histogram gradient boosting (extension nuisance learner; BASELINE config 5,
SURVEY.md K11-K14 + C04).

``fit_gbdt`` grows depth-limited trees level by level on the binned uint8 panel:
GPU (csrc/gbdt.hip) or the numpy reference (reference/gbdt.py) — same spec, same
integer histogram sums, so the same trees. With ``dist`` (row shards), each level's
compact node histograms are all-reduced (C04, exact int64) on the fit's stream between
steps of the native level loop (``ate_gbdt_run``) -- at world W > 1 reduce-scattered by
feature slice, each rank searching its slice and the per-block split candidates
all-gathered (``c04_slices``) -- and every rank takes the same split decisions; the base score is an exact fixed-point mean and the bin edges come from a
GLOBAL row sample (``global_bin_edges``), so a row-sharded fit grows the same trees bit
for bit at every world size.
"""
from __future__ import annotations

import ctypes
import os
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
    scores: object = None  # raw boosting score of every row seen in training (train or not)

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
        """Xb: column-major [p][n] bins (models/forest.py::bin_matrix)."""
        n = Xb.shape[1]
        if self.backend == "gpu":
            Xr, ldr = _to_rowmajor(Xb)
            f = torch.full((n,), self.base, dtype=torch.float64, device=Xb.device)
            M = self.feat.shape[1]
            _native.call("ate_gbdt_apply", Xr.data_ptr(), ldr, n, self.n_trees, M,
                         self.feat.data_ptr(), self.thr.data_ptr(), self.value.data_ptr(),
                         f.data_ptr(), torch.cuda.current_stream().cuda_stream)
            return f.cpu().numpy()
        Xn = Xb.numpy() if isinstance(Xb, torch.Tensor) else Xb
        t = ref.GbdtTrees(np.asarray(self.feat), np.asarray(self.thr), np.asarray(self.value),
                          self.base, self.loss, self.depth)
        return t.predict_binned(Xn)


EDGE_SAMPLE = 200_000


def sample_bin_edges(X, rows=EDGE_SAMPLE, device=None):
    """Quantile edges from an evenly strided row sample when n is large (the standard
    histogram-GBDT construction; exact for features with <= 256 distinct values in it).
    With a GPU ``device`` the sort runs there (models/forest.py::bin_edges_device, same
    edges bit for bit)."""
    X = np.asarray(X, dtype=np.float64)
    n = X.shape[0]
    if n > rows:
        X = X[np.linspace(0, n - 1, num=rows).astype(np.int64)]
    if device is not None and torch.device(device).type == "cuda":
        return F.bin_edges_device(torch.as_tensor(X, device=device))
    return F.bin_edges(X)


def binned(X, edges, device):
    """Binned panel for fit_gbdt(Xb=...): device row-major [n][ldr] (ldr % 32 == 0, the
    layout of csrc/gbdt.hip) or host column-major [p][n] (the numpy reference's)."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if dev.type == "cuda":
        return _rowmajor_bins(X, edges, dev)
    Xb = F.bin_matrix(np.asarray(X, dtype=np.float64), edges[0], edges[1], None).numpy()
    return Xb, Xb.shape[1]


def _to_rowmajor(Xb):
    """[p][n] column-major bins -> [n][ldr] row-major, ldr = p rounded up to 32."""
    p, n = Xb.shape
    ldr = -(-p // 32) * 32
    out = torch.zeros((n, ldr), dtype=torch.uint8, device=Xb.device)
    out[:, :p] = Xb.t()
    return out, ldr


def _rowmajor_bins(X, edges, dev):
    return _to_rowmajor(F.bin_matrix(np.asarray(X, dtype=np.float64), edges[0], edges[1], dev))


def global_sample_ids(n_total, rows=EDGE_SAMPLE):
    """Global row ids of the bin-edge sample: evenly strided over ALL rows (the single-
    device ``sample_bin_edges`` rows), so the edges do not depend on the sharding."""
    if n_total <= rows:
        return np.arange(n_total, dtype=np.int64)
    return np.linspace(0, n_total - 1, num=rows).astype(np.int64)


def global_bin_edges(X_local, dist, rows=EDGE_SAMPLE, device=None):
    """Bin edges every rank agrees on, EQUAL to the single-device edges: each rank
    contributes its rows of the global strided sample (global_sample_ids), the pieces are
    all-gathered in rank order (= global row order) and binned together."""
    X_local = np.asarray(X_local, dtype=np.float64)
    if dist is None or dist.world == 1:
        return sample_bin_edges(X_local, rows=rows, device=device)
    from ..parallel.dist import shard_range
    ids = global_sample_ids(dist.n_total, rows)
    mine = ids[(ids >= dist.row_offset) & (ids < dist.row_offset + dist.n_local)] - dist.row_offset
    counts = [int(((ids >= o) & (ids < o + m)).sum())
              for o, m in (shard_range(dist.n_total, r, dist.world) for r in range(dist.world))]
    on_dev = device is not None and torch.device(device).type == "cuda" and \
        bool(getattr(dist.comm, "capturable", False))          # RCCL gathers device tensors
    s = torch.zeros((max(counts), X_local.shape[1]), dtype=torch.float64,
                    device=device if on_dev else "cpu")
    s[:len(mine)] = torch.as_tensor(X_local[mine], device=s.device)
    parts = dist.comm.all_gather(s)
    S = torch.cat([pp[:c] for pp, c in zip(parts, counts)])
    if device is not None and torch.device(device).type == "cuda":
        return F.bin_edges_device(S.to(device))
    return F.bin_edges(S.cpu().numpy())


def fit_gbdt(X, y, loss="squared", n_trees=100, depth=6, lr=0.1, lam=1.0, min_child=1.0,
             min_gain=0.0, train=None, backend=None, edges=None, dist=None, seed=0,
             Xb=None) -> GbdtModel:
    """X [n, p] float, y [n]; ``train`` (bool [n]) restricts the rows the trees learn
    from; ``model.scores`` holds the final raw score of EVERY row (so held-out
    predictions come for free). ``Xb=(binned, ld)`` from ``binned()`` reuses one binned
    panel across fits (X and edges are then only used for bookkeeping). ``seed`` is
    reserved for row/column subsampling (not used: full-data boosting is deterministic)."""
    on_dev = isinstance(y, torch.Tensor) and y.is_cuda
    if not on_dev:
        y = np.asarray(y.cpu() if isinstance(y, torch.Tensor) else y, dtype=np.float64)
    if Xb is None:
        X = np.asarray(X, dtype=np.float64)
        n, p = X.shape
    else:
        n = len(y)
        p = Xb[0].shape[0] if isinstance(Xb[0], np.ndarray) or Xb[0].device.type == "cpu" \
            else len(edges[0])
    if depth < 1 or depth > MAX_DEPTH:
        raise ValueError(f"depth must be in [1, {MAX_DEPTH}] (<= {2 ** (MAX_DEPTH - 1)} nodes "
                         "per level histogram, csrc/gbdt.hip MAXD)")
    if backend is None:
        backend = "gpu" if torch.cuda.is_available() else "cpu"
    if edges is None:
        edges = global_bin_edges(X, dist)
    if train is None:
        train = torch.ones(n, dtype=torch.bool, device=y.device) if on_dev else \
            np.ones(n, dtype=bool)
    elif not on_dev:
        train = np.asarray(train.cpu() if isinstance(train, torch.Tensor) else train, dtype=bool)
    if backend != "gpu":
        if Xb is None:
            Xbh = F.bin_matrix(X, edges[0], edges[1], None).numpy()
        elif isinstance(Xb[0], torch.Tensor) and Xb[0].device.type == "cuda":
            Xbh = Xb[0][:, :p].t().cpu().numpy()          # device row-major panel
        else:
            Xbh = np.asarray(Xb[0].cpu() if isinstance(Xb[0], torch.Tensor) else Xb[0])
        red = c04 = None
        if dist is not None and dist.world > 1:
            def red(a):
                t = torch.from_numpy(np.ascontiguousarray(a))
                return dist.sum_(t).numpy()
            nr, pw = c04_slices(p, dist)
            if nr > 1:
                c04 = SlicedC04(dist, p, nr, pw)
        tr = ref.fit(Xbh, y, train, loss, n_trees, depth, lr, lam, min_child, min_gain,
                     hist_reduce=red, c04=c04)
        return GbdtModel(tr.feat, tr.thr, tr.value, tr.base, loss, depth, edges, "cpu",
                         tr.predict_binned(Xbh))
    dev = torch.device("cuda", torch.cuda.current_device())
    _check_limits()
    Xr, ldr = Xb if Xb is not None else _rowmajor_bins(X, edges, dev)
    return _fit_gpu(Xr, ldr, p, y, train, loss, n_trees, depth, lr, lam, min_child, min_gain,
                    edges, dist, dev)


MAX_DEPTH = 8      # csrc/gbdt.hip MAXD
_limits_ok = False


def _check_limits():
    """The buffers below are sized with MAX_DEPTH / MAXB; the kernels index them with the
    library's own compile-time limits: refuse to run on a mismatched build."""
    global _limits_ok
    if _limits_ok:
        return
    out = (ctypes.c_int * 3)()
    _native.call("ate_gbdt_limits", ctypes.cast(out, ctypes.c_void_p))
    if (out[0], out[1]) != (MAX_DEPTH, MAXB):
        raise RuntimeError(f"libatehip GBDT limits (MAXD {out[0]}, MAXB {out[1]}) differ from "
                           f"models/gbdt.py (MAX_DEPTH {MAX_DEPTH}, MAXB {MAXB}): rebuild")
    _limits_ok = True


class FitArgs(ctypes.Structure):
    """Mirror of csrc/gbdt.hip::GbdtFitArgs."""
    P = ctypes.c_void_p
    _fields_ = [("Xr", P), ("ldr", ctypes.c_int64), ("n", ctypes.c_int64),
                ("n_train", ctypes.c_int64), ("p", ctypes.c_int), ("depth", ctypes.c_int),
                ("n_trees", ctypes.c_int), ("loss", ctypes.c_int), ("rule", ctypes.c_int),
                ("W", ctypes.c_int), ("lam", ctypes.c_double), ("min_gain", ctypes.c_double),
                ("lr", ctypes.c_double), ("min_child", ctypes.c_int64), ("R", ctypes.c_int64),
                ("y", P), ("f", P), ("idx", P * 2), ("gh", P * 2), ("bkt", P), ("cnt", P),
                ("base", P), ("btot", P), ("seg", P * 2), ("tot", P), ("feat", P), ("thr", P),
                ("value", P), ("H", P * 2), ("Hs", P), ("slab", P), ("slab_cap", ctypes.c_int64),
                ("cand", P), ("nr", ctypes.c_int), ("rk", ctypes.c_int), ("pw", ctypes.c_int),
                ("pl", ctypes.c_int), ("Hl", P), ("candg", P)]


class RunState(ctypes.Structure):
    """Mirror of csrc/gbdt.hip::GbdtRunState (resumable position of a fit; t_stop > 0 ends
    the run after tree t_stop - 1, for the lockstep pair fits)."""
    _fields_ = [("t", ctypes.c_int), ("d", ctypes.c_int), ("cur", ctypes.c_int),
                ("resume", ctypes.c_int), ("red_count", ctypes.c_int64), ("t_stop", ctypes.c_int)]


MAXB = 2 ** (MAX_DEPTH - 1) + 1    # csrc/gbdt.hip MAXB: partition buckets + retired


def c04_slices(p, dist):
    """Feature-sliced C04 geometry (nr, pw): nr rank blocks of pw = ceil(p / nr) features
    (rank r owns [r * pw, min(p, r * pw + pw))), or (1, p) for a single device, when
    ATE_GBDT_C04=allreduce, or when some rank's slice would be empty (p small next to
    the world size)."""
    if dist is None or dist.world == 1 or os.environ.get("ATE_GBDT_C04", "") == "allreduce":
        return 1, p
    w = dist.world
    pw = -(-p // w)
    if p - (w - 1) * pw < 1:
        return 1, p
    return w, pw


class SlicedC04:
    """Feature-sliced C04 for the numpy reference fit (reference/gbdt.fit ``c04``): the
    scheme of the device stepper (csrc/gbdt.hip header) with host collectives."""

    def __init__(self, dist, p, nr, pw):
        self.dist, self.p, self.nr, self.pw = dist, p, nr, pw
        self.joff = dist.rank * pw
        self.pl = min(pw, p - self.joff)

    def scatter(self, hist):
        nn = hist.shape[0]
        img = np.zeros((nn, self.nr * self.pw, 256, 2), dtype=np.int64)
        img[:, :self.p] = hist
        # rank-block-major [nr][nn][pw][256][2]: rank r's reduce-scatter chunk is its slice
        t = torch.from_numpy(np.ascontiguousarray(
            img.reshape(nn, self.nr, self.pw, 256, 2).transpose(1, 0, 2, 3, 4))).reshape(-1)
        out = torch.empty(t.numel() // self.nr, dtype=torch.int64)
        self.dist.comm.reduce_scatter_(out, t)
        return out.numpy().reshape(nn, self.pw, 256, 2)[:, :self.pl]

    def pick(self, sps):
        nn = len(sps)
        c = np.zeros((nn, 5), dtype=np.int64)
        c[:, 0] = np.float64(-np.inf).view(np.int64)
        for k, sp in enumerate(sps):
            if sp is not None:
                c[k] = [np.float64(sp[0]).view(np.int64), *sp[1:]]
        g = torch.empty(self.nr * c.size, dtype=torch.int64)
        self.dist.comm.all_gather_into_(g, torch.from_numpy(c.reshape(-1)))
        g = g.numpy().reshape(self.nr, nn, 5)
        out = []
        for k in range(nn):
            best = None
            for r in range(self.nr):
                gain = float(g[r, k, 0].view(np.float64))
                if gain == -np.inf:
                    continue
                key = (-gain, int(g[r, k, 1]), int(g[r, k, 2]))
                if best is None or key < best[0]:
                    best = (key, (gain, *(int(v) for v in g[r, k, 1:])))
            out.append(None if best is None else best[1])
        return out


def exact_base(y_train, n_train, loss, dist=None):
    """Base score from the EXACT sum of the training targets (2^-28 fixed point, as the
    histograms): identical bits for any row sharding (reference/gbdt.base_score)."""
    if isinstance(y_train, torch.Tensor):
        ys = torch.round(y_train.double() * ref.FIX).to(torch.int64).sum().reshape(1)
    else:
        ys = torch.tensor([int(ref.fix(y_train).sum())], dtype=torch.int64)
    cnt = torch.cat([ys, torch.tensor([int(n_train)], dtype=torch.int64, device=ys.device)])
    if dist is not None:
        dist.sum_(cnt)
    c = cnt.cpu()
    return ref.base_from_sums(int(c[0]), int(c[1]), loss)


def _fit_gpu(Xr, ldr, p, y, train, loss, n_trees, depth, lr, lam, min_child, min_gain, edges,
             dist, dev):
    """y: [n] targets, train: [n] bool (numpy or device tensors: the HBM-panel path keeps
    them on the device)."""
    fs = _GpuFit(Xr, ldr, p, y, train, loss, n_trees, depth, lr, lam, min_child, min_gain,
                 edges, dist, dev)
    if not fs.empty:
        fs.drive(dist)
    return fs.model()


class _GpuFit:
    """One device fit: its buffers, the native argument block (csrc/gbdt.hip GbdtFitArgs)
    and the stepper position. ``slab_min``: slab entries to allocate at least (the fused
    root pass of fit_gbdt_pair writes fit A's slab)."""

    def __init__(self, Xr, ldr, p, y, train, loss, n_trees, depth, lr, lam, min_child,
                 min_gain, edges, dist, dev, slab_min=0):
        yt = torch.as_tensor(y, device=dev, dtype=torch.float64)
        trn = torch.as_tensor(train, device=dev, dtype=torch.bool)
        n = yt.numel()
        order = torch.cat([torch.nonzero(trn).flatten(), torch.nonzero(~trn).flatten()])
        n_train = int(trn.sum())
        base = exact_base(yt[order[:n_train]], n_train, loss, dist)
        M = 2 ** (depth + 1) - 1
        self.loss, self.depth, self.edges, self.base, self.n_train = loss, depth, edges, base, n_train
        self.f = torch.full((n,), base, dtype=torch.float64, device=dev)
        self.feat = torch.full((n_trees, M), -2, dtype=torch.int32, device=dev)
        self.thr = torch.zeros((n_trees, M), dtype=torch.int32, device=dev)
        self.value = torch.zeros((n_trees, M), dtype=torch.float64, device=dev)
        self.empty = n_train == 0 or n_trees == 0
        if self.empty:
            # a rank may hold no training rows; it still has to join every collective
            if dist is not None and dist.world > 1 and n_trees:
                raise ValueError("row-sharded GBDT needs training rows on every rank")
            return
        i32 = dict(dtype=torch.int32, device=dev)
        i64 = dict(dtype=torch.int64, device=dev)
        R = max(1024, -(-n_train // 1024))
        R = -(-R // 256) * 256
        W = -(-n_train // R)
        self.idx = [order[:n_train].to(torch.int32).contiguous(), torch.empty(n_train, **i32)]
        self.gh = [torch.empty(n_train, **i64), torch.empty(n_train, **i64)]
        self.yt, self.bkt = yt, torch.empty(n_train, dtype=torch.uint8, device=dev)
        self.cntb = torch.empty(MAXB * W, **i32)
        self.baseb = torch.empty(MAXB * W, **i32)
        self.btot = torch.empty(MAXB, **i32)
        self.seg = [torch.zeros(MAXB + 1, **i32), torch.zeros(MAXB + 1, **i32)]
        self.tot = torch.zeros(2 * M, **i64)
        # rule 1 (hessian child rule + a pause per level for the histogram all-reduce) for
        # every row-sharded fit, world 1 included (the same code path as world W)
        rule = 0 if dist is None else 1
        # world W > 1: feature-sliced C04 (reduce-scatter of the level histograms, split
        # search on this rank's pw features, all-gather of the candidates; csrc/gbdt.hip)
        nr, pw = c04_slices(p, dist) if rule == 1 else (1, p)
        self.nr, self.pw, self.rule = nr, pw, rule
        rk = dist.rank if nr > 1 else 0
        slots = max(1, 2 ** (depth - 2))
        self.H = [torch.empty(2 ** (depth - 1) * 512 * pw, **i64) for _ in range(2)]
        self.Hs = torch.empty(slots * 512 * nr * pw, **i64)
        self.Hl = torch.empty(slots * 512 * pw, **i64) if nr > 1 else None
        cap = max(int(_native.hip().ate_gbdt_slab_entries(n_train, p, depth, rule)), int(slab_min))
        self.slab = torch.empty(cap, **i64)
        ncand = (1 << max(depth - 1, 0)) * (-(-pw // 8)) * 4                 # 32-B Cand
        self.cand = torch.empty(ncand, **i64)
        self.candg = torch.empty(nr * ncand, **i64) if nr > 1 else None
        P = ctypes.c_void_p
        a = FitArgs(Xr=Xr.data_ptr(), ldr=ldr, n=n, n_train=n_train, p=p, depth=depth,
                    n_trees=n_trees, loss=LOSS[loss], rule=rule, W=W, lam=lam,
                    min_gain=min_gain, lr=lr, min_child=int(np.rint(min_child * ref.FIX)), R=R,
                    y=yt.data_ptr(), f=self.f.data_ptr(), bkt=self.bkt.data_ptr(),
                    cnt=self.cntb.data_ptr(), base=self.baseb.data_ptr(),
                    btot=self.btot.data_ptr(), tot=self.tot.data_ptr(),
                    feat=self.feat.data_ptr(), thr=self.thr.data_ptr(),
                    value=self.value.data_ptr(), Hs=self.Hs.data_ptr(),
                    slab=self.slab.data_ptr(), slab_cap=cap, cand=self.cand.data_ptr(),
                    nr=nr, rk=rk, pw=pw, pl=min(pw, p - rk * pw),
                    Hl=self.Hl.data_ptr() if self.Hl is not None else None,
                    candg=self.candg.data_ptr() if self.candg is not None else None)
        a.idx = (P * 2)(self.idx[0].data_ptr(), self.idx[1].data_ptr())
        a.gh = (P * 2)(self.gh[0].data_ptr(), self.gh[1].data_ptr())
        a.seg = (P * 2)(self.seg[0].data_ptr(), self.seg[1].data_ptr())
        a.H = (P * 2)(self.H[0].data_ptr(), self.H[1].data_ptr())
        self.a, self.st = a, RunState()

    def model(self):
        return GbdtModel(self.feat, self.thr, self.value, self.base, self.loss, self.depth,
                         self.edges, "gpu", self.f)

    def drive(self, dist):
        """Run the stepper from its position until it returns 0, servicing the row-sharded
        fit's pauses: level histograms all-reduced (C04) -- or, feature-sliced, reduce-
        scattered, and after the slice's split search the candidates all-gathered -- on the
        same stream (no host callback, no host sync)."""
        a, st, nr = self.a, self.st, self.nr
        run = _native.hip().ate_gbdt_run
        while True:
            rc = run(ctypes.addressof(a), ctypes.addressof(st),
                     ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
            if rc == 0:
                break
            if rc not in (1, 2) or dist is None or (rc == 2 and nr == 1):
                raise RuntimeError(f"ate_gbdt_run failed with status {rc}")
            self.reduce(dist, rc, st.red_count)

    def reduce(self, dist, rc, m):
        if rc == 1 and self.nr == 1:
            dist.sum_(self.Hs[:m])
        elif rc == 1:
            dist.comm.reduce_scatter_(self.Hl[:m // self.nr], self.Hs[:m])
        else:
            dist.comm.all_gather_into_(self.candg[:self.nr * m], self.cand[:m])


# Lockstep pair fits with a fused root histogram pass (fit_gbdt_pair); ATE_GBDT_FUSED_ROOT=0
# fits a pair one after the other (the A/B of profiles/r06_cfg5)
FUSED_ROOT = os.environ.get("ATE_GBDT_FUSED_ROOT", "1") == "1"


def _two_ranges(rows):
    """(a0, n0, a1) when the ascending row list ``rows`` is rows a0 .. a0 + n0 - 1 followed by
    a1, a1 + 1, ... (a fold's complement on a fold-segmented panel), else (0, -1, 0): the
    fused root pass then computes each position's row instead of loading it."""
    n = rows.numel()
    if n == 0:
        return 0, -1, 0
    brk = torch.nonzero(rows[1:] - rows[:-1] != 1).flatten()
    if brk.numel() > 1:
        return 0, -1, 0
    n0 = int(brk[0]) + 1 if brk.numel() else n
    return int(rows[0]), n0, int(rows[n0]) if n0 < n else int(rows[0]) + n0


def fit_gbdt_pair(ys, losses, train, Xb, edges, dist=None, n_trees=100, depth=6, lr=0.1,
                  lam=1.0, min_child=1.0, min_gain=0.0):
    """Two device fits on the SAME training rows and binned panel -- a DML fold's E[Y|X] and
    E[W|X] (estimators/boosting._crossfit) -- in lockstep, tree by tree. Level 0 of both trees
    comes from ONE pass over the rows' bins (csrc/gbdt.hip ate_gbdt_pair_root: four-channel
    LDS histograms, gbdt_hist2_kernel); levels 1.. and the score walk are each fit's own
    stepper. Every histogram is an exact integer sum, so the trees, scores and held-out
    predictions are the bits of two fit_gbdt calls (tests/test_gbdt_gpu.py). With ``dist``
    each fit's root histogram is all-reduced / reduce-scattered (C04) as in the stepper.
    Returns the two GbdtModels."""
    dev = torch.device("cuda", torch.cuda.current_device())
    _check_limits()
    Xr, ldr = Xb
    p = len(edges[0])
    if depth < 1 or depth > MAX_DEPTH:
        raise ValueError(f"depth must be in [1, {MAX_DEPTH}]")
    trn = torch.as_tensor(train, device=dev, dtype=torch.bool)
    n_train = int(trn.sum())
    cap2 = int(_native.hip().ate_gbdt_slab2_entries(max(n_train, 1), p)) if n_train else 0
    fits = [_GpuFit(Xr, ldr, p, ys[0], trn, losses[0], n_trees, depth, lr, lam, min_child,
                    min_gain, edges, dist, dev, slab_min=cap2),
            _GpuFit(Xr, ldr, p, ys[1], trn, losses[1], n_trees, depth, lr, lam, min_child,
                    min_gain, edges, dist, dev)]
    A, B = fits
    if A.empty or B.empty:
        for fs in fits:
            if not fs.empty:
                fs.drive(dist)
        return A.model(), B.model()
    idx_root = A.idx[0].clone()          # the training rows in row order (any order: same trees)
    gh2 = torch.empty(2 * A.n_train, dtype=torch.int64, device=dev)
    a0, n0, a1 = _two_ranges(idx_root)
    for t in range(n_trees):
        s = torch.cuda.current_stream().cuda_stream
        _native.call("ate_gbdt_pair_root", ctypes.addressof(A.a), ctypes.addressof(B.a),
                     idx_root.data_ptr(), gh2.data_ptr(), a0, n0, a1, s)
        for fs in fits:
            if fs.rule == 1:                 # the root's compact histogram (C04)
                fs.reduce(dist, 1, 512 * fs.nr * fs.pw)
            fs.st.t, fs.st.d, fs.st.cur, fs.st.resume, fs.st.t_stop = t, 0, 0, 1, t + 1
            fs.drive(dist)
    return A.model(), B.model()
