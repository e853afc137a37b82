"""Forest nuisance learners on the binned-histogram engine.

* ``rf_classifier`` — randomForest semantics used by ``doubly_robust`` and
  ``chernozhukov`` (``ate_functions.R:169-174,340-357``): bootstrap, mtry =
  floor(sqrt(p)), nodesize 1, Gini, majority-vote leaves, ``predict(type="prob")`` =
  vote share, OOB votes when predicting the training rows.
* ``regression_forest`` / ``causal_forest`` — grf semantics
  (``ate_replication.Rmd:250-265``): little bags of 2 trees on half-samples, honesty,
  min.node.size 5, alpha 0.05, mtry = min(ceil(sqrt(p)+20), p) drawn ~ Poisson,
  causal splits on gradient pseudo-outcomes, leaf sufficient statistics (forest
  weights without N^2 storage), OOB predictions and little-bag variance.

Backends: ``"gpu"`` (csrc/forest.hip, one workgroup per tree) and ``"cpu"``
(csrc/cpu/forest_cpu.cpp, OpenMP). Both implement the spec in
csrc/forest_common.hpp and grow bit-identical trees from the same Philox streams.
Continuous covariates are quantile-binned to <= 256 bins (exact for <= 256 distinct
values); splits are at bin boundaries.

Exact-split mode (``splits="exact"``): bins are the ranks of every feature's distinct
values (uint16, <= 65536 rows), splits can fall between any two consecutive distinct
in-node values. randomForest (bootstrap, kinds 0/1): the threshold is their midpoint
(``findbestsplit``); grf (half-samples, honesty, little bags; kinds 1/2): the left value
itself (x <= v goes left), so new rows are binned by #{values < x}. GPU:
csrc/forest_exact.hip, host twin grow_tree_exact in csrc/cpu/forest_cpu.cpp -- the same
trees bit for bit. ``splits="auto"`` picks exact splits up to 65,536 rows (the tutorial's
scale, where randomForest and grf themselves split on exact values).
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass

import numpy as np
import torch

from .. import _native

MAX_BINS = 256


class ForestParams(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("sampling", ctypes.c_int), ("ntree", ctypes.c_int),
                ("mtry", ctypes.c_int), ("min_node", ctypes.c_int), ("honesty", ctypes.c_int),
                ("group", ctypes.c_int), ("mtry_poisson", ctypes.c_int),
                ("alpha", ctypes.c_double), ("sample_fraction", ctypes.c_double),
                ("pois0", ctypes.c_double), ("seed", ctypes.c_uint64), ("p", ctypes.c_int),
                ("n", ctypes.c_int), ("t0", ctypes.c_int)]


KIND_CLASS, KIND_REG, KIND_CAUSAL = 0, 1, 2
FIX = float(2 ** 32)
# causal-split admissibility rule the engines implement (part of checkpoint keys):
# grf stabilize.splits=TRUE -- each child holds >= max(ceil(alpha n), 1) rows on both sides
# of the node's mean centred treatment (csrc/forest_common.hpp)
CAUSAL_SPLIT_RULE = "grf-stabilize"


def to_fix(v) -> np.ndarray:
    """2^-32 fixed point, round half away from zero (forest_common.hpp::to_fix)."""
    s = np.asarray(v, dtype=np.float64) * FIX
    return np.where(s >= 0, np.floor(s + 0.5), np.ceil(s - 0.5)).astype(np.int64)


def from_fix(v) -> np.ndarray:
    return np.asarray(v, dtype=np.float64) / FIX


# ------------------------------------------------------------------ K11 binning
DEVICE_EDGES_MIN = 1 << 21   # n * p from which a GPU fit sorts for its edges on the device
def bin_edges(X: np.ndarray, max_bins: int = MAX_BINS):
    """Per-feature sorted edges (<= max_bins-1): midpoints between distinct values when
    there are at most max_bins of them, else distinct quantiles."""
    X = np.asarray(X, dtype=np.float64)
    p = X.shape[1]
    edges = np.full((p, MAX_BINS - 1), np.inf)
    ne = np.zeros(p, dtype=np.int32)
    for j in range(p):
        u = np.unique(X[:, j])
        if len(u) <= max_bins:
            e = (u[:-1] + u[1:]) / 2.0
        else:
            qs = np.quantile(X[:, j], np.arange(1, max_bins) / max_bins, method="lower")
            e = np.unique(qs)
            e = e[e < u[-1]]
        edges[j, :len(e)] = e
        ne[j] = len(e)
    return edges, ne


def bin_edges_device(X: torch.Tensor, max_bins: int = MAX_BINS):
    """``bin_edges`` with the sorting on the device (X: [n, p] float64 tensor). Same
    semantics, same bits: midpoints of the distinct values, else numpy's
    ``quantile(method="lower")`` order statistics sorted[(n-1) k // max_bins]."""
    n, p = X.shape
    S = torch.sort(X.double(), dim=0).values                    # [n, p]
    ndist = ((S[1:] != S[:-1]).sum(0) + 1).cpu().numpy() if n > 1 else np.ones(p, np.int64)
    qi = torch.as_tensor([(n - 1) * k // max_bins for k in range(1, max_bins)],
                         device=X.device)
    Q = S.index_select(0, qi).t().cpu().numpy()                 # [p, max_bins-1]
    top = S[-1].cpu().numpy()
    edges = np.full((p, MAX_BINS - 1), np.inf)
    ne = np.zeros(p, dtype=np.int32)
    for j in range(p):
        if ndist[j] <= max_bins:
            u = torch.unique_consecutive(S[:, j]).cpu().numpy()
            e = (u[:-1] + u[1:]) / 2.0
        else:
            e = np.unique(Q[j])
            e = e[e < top[j]]
        edges[j, :len(e)] = e
        ne[j] = len(e)
    return edges, ne


def bin_matrix(X, edges, ne, device=None) -> torch.Tensor:
    """uint8 [p][n] column-major bins: bin(x) = #{edges < x}."""
    Xn = X if isinstance(X, torch.Tensor) else torch.as_tensor(np.asarray(X, dtype=np.float64))
    n, p = Xn.shape
    dev = torch.device("cpu") if device is None else torch.device(device)
    if dev.type == "cuda":
        Xc = Xn.to(dev, torch.float64).t().contiguous()
        out = torch.empty((p, n), dtype=torch.uint8, device=dev)
        e = torch.as_tensor(edges, device=dev, dtype=torch.float64).contiguous()
        nt = torch.as_tensor(ne, device=dev, dtype=torch.int32)
        _native.call("ate_bin_matrix", Xc.data_ptr(), n, p, e.data_ptr(), nt.data_ptr(),
                     out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        return out
    Xh = Xn.double().cpu().numpy()
    out = np.empty((p, n), dtype=np.uint8)
    for j in range(p):
        out[j] = np.searchsorted(edges[j, :ne[j]], Xh[:, j], side="left")
    return torch.from_numpy(out)


EXACT_MAX_ROWS = 65536


@dataclass
class ExactBins:
    """Value-rank binning of the exact-split mode: vals [p][ldv] sorted distinct values
    (+inf padded), nval [p] their counts, mids [p][ldv-1] midpoints between consecutive
    values (bin(x) = #{mids < x}: the rank of x when x is in the table)."""
    vals: np.ndarray
    nval: np.ndarray
    mids: np.ndarray

    @property
    def ldv(self):
        return self.vals.shape[1]

    def on(self, dev) -> "DeviceExactBins":
        """The value table as device tensors (inputs of a captured estimator graph)."""
        return DeviceExactBins(torch.as_tensor(self.vals, device=dev),
                               torch.as_tensor(self.nval, device=dev))

    def bin(self, X, grf: bool = False) -> np.ndarray:
        """uint16 [p][n] column-major bins of X (host): #{midpoints < x} (randomForest's
        midpoint thresholds) or, ``grf``, #{values < x} (grf's x <= value rule). Both are
        the value's rank for a value in the table."""
        Xh = np.asarray(X.detach().cpu().numpy() if isinstance(X, torch.Tensor) else X,
                        dtype=np.float64)
        p = self.vals.shape[0]
        out = np.empty((p, Xh.shape[0]), dtype=np.uint16)
        for j in range(p):
            ref = self.vals[j, :self.nval[j]] if grf else self.mids[j, :self.nval[j] - 1]
            out[j] = np.minimum(np.searchsorted(ref, Xh[:, j], side="left"),
                                self.nval[j] - 1)
        return out


@dataclass
class DeviceExactBins:
    """ExactBins.vals / nval resident on the device (no host data: rows must come binned)."""
    vals: torch.Tensor
    nval: torch.Tensor

    @property
    def ldv(self):
        return self.vals.shape[1]

    def bin(self, X):
        raise ValueError("a device-only exact bin table cannot bin new rows; pass binned rows")


# "auto" keeps exact splits only while a tree's per-feature row lists stay small: the exact
# engine's scratch holds two [p][in-bag rows] uint32 lists per tree (csrc/forest_exact.hip
# tree_bytes), 8 p n bytes -- 5 MB at the tutorial's p = 21, n = 3e4, but 268 MB per tree at
# p = 512, n = 65,536, where a 1-GiB launch cap would hold ~3 trees.
EXACT_AUTO_LIST_BYTES = 64 << 20


def exact_list_bytes(n: int, p: int) -> int:
    """Bytes of a tree's two per-feature row lists in the exact engine (in-bag rows <= n)."""
    return 8 * int(p) * int(n)


def resolve_splits(splits: str, n: int, p: int | None = None) -> str:
    """"auto": randomForest's exact splits when the rows fit the uint16 value ranks
    (n <= 65536, the tutorial scale) and, given ``p``, a tree's row lists fit
    ``EXACT_AUTO_LIST_BYTES``; else the 256-bin histogram engine."""
    if splits == "auto":
        if n > EXACT_MAX_ROWS:
            return "binned"
        if p is not None and exact_list_bytes(n, p) > EXACT_AUTO_LIST_BYTES:
            return "binned"
        return "exact"
    if splits not in ("binned", "exact"):
        raise ValueError(f"splits must be 'auto', 'binned' or 'exact', got {splits!r}")
    return splits


def exact_bins(X) -> ExactBins:
    """Distinct values of every feature of X (n <= 65536 rows)."""
    X = np.asarray(X.detach().cpu().numpy() if isinstance(X, torch.Tensor) else X,
                   dtype=np.float64)
    n, p = X.shape
    if n > EXACT_MAX_ROWS:
        raise ValueError(f"exact-split forests take at most {EXACT_MAX_ROWS} rows (got {n})")
    us = [np.unique(X[:, j]) for j in range(p)]
    ldv = max(2, max(len(u) for u in us))
    vals = np.full((p, ldv), np.inf)
    mids = np.full((p, ldv - 1), np.inf)
    nval = np.zeros(p, dtype=np.int32)
    for j, u in enumerate(us):
        vals[j, :len(u)] = u
        mids[j, :len(u) - 1] = (u[:-1] + u[1:]) / 2.0
        nval[j] = len(u)
    return ExactBins(vals, nval, mids)


# ------------------------------------------------------------------ forest object
def _nthreads():
    return int(os.environ.get("ATE_CPU_THREADS", os.cpu_count() or 1))


@dataclass
class Forest:
    params: ForestParams
    backend: str
    cap: int
    feat: object
    thr: object
    left: object
    val: object
    nnodes: object
    inbag: object
    est: object
    edges: np.ndarray
    nedges: np.ndarray
    Xb_train: object = None
    packed: object = None        # GPU: int2 per node (see csrc/forest.hip forest_pack_kernel)
    exact: ExactBins | None = None   # exact-split forests: uint16 value-rank bins
    # GPU exact-split fits: (device count of trees with nnodes = -1, ntree, mc), checked at the
    # first host read (check()), so that the fit itself never waits for the device
    overflow: object = None

    def check(self):
        """Raise if the exact-split fit flagged trees whose in-bag count exceeded the host's
        bound mc (csrc/forest_exact.hip sets nnodes = -1; exact_mcap is exact, so never
        expected). Runs once, at the first host read of the forest's outputs."""
        if self.overflow is None:
            return
        cnt, ntree, mc = self.overflow
        self.overflow = None
        bad = int(cnt)
        if bad:
            raise RuntimeError(f"exact forest: {bad} of {ntree} trees overflowed the in-bag "
                               f"bound mc = {mc} (models/forest.exact_mcap)")

    @property
    def device(self):
        return torch.device("cuda", torch.cuda.current_device()) if self.backend == "gpu" \
            else torch.device("cpu")

    def _bins(self, X):
        if X is None:
            return self.Xb_train
        if self.exact is not None:
            b = torch.from_numpy(self.exact.bin(X, grf=self.params.sampling == 1))
            return b.to(self.device) if self.backend == "gpu" else b
        dev = self.device if self.backend == "gpu" else None
        return bin_matrix(X, self.edges, self.nedges, dev)

    def predict_raw(self, X=None, oob=False) -> np.ndarray:
        """kind 0/1: [n] predictions; kind 2: [n, 4] (tau, var, trees used, groups used)."""
        Xb = self._bins(X)
        state = self.new_state(Xb.shape[1])
        return self.predict_state(Xb, oob, state, phases=7)

    def new_state(self, n2):
        """Prediction accumulators [10, n2]: int64 sums of per-tree terms in 2^-32 fixed
        point (csrc/forest_common.hpp mean_fix) -- exact and order-free, so tree-parallel
        ranks all-reduce them to the single-device bits."""
        if self.backend == "gpu":
            return torch.zeros(10 * n2, dtype=torch.int64, device=self.device)
        return np.zeros(10 * n2, dtype=np.int64)

    def predict_state(self, Xb, oob, state, phases, host=True):
        """Run prediction phases (1: per-tree sums, 2: little-bag group sums, 4: finalise)
        on accumulator ``state`` ([10, n2]); returns the predictions when phase 4 ran
        (``host=False``, GPU: the device tensor, no host sync -- capturable)."""
        n2 = Xb.shape[1]
        if oob and n2 != self.params.n:
            raise ValueError("OOB prediction requires the training rows")
        width = 4 if self.params.kind == KIND_CAUSAL else 1
        if self.backend == "gpu":
            dev = self.device
            s = torch.cuda.current_stream().cuda_stream
            if self.exact is not None:
                # trees per chunk rounded to the little-bag group BEFORE sizing the leaf
                # buffer (a 1-tree chunk of a group-2 forest becomes 2 trees)
                g = max(1, self.params.group) if self.params.kind == KIND_CAUSAL else 1
                tchunk = max(g, min(self.params.ntree, (1 << 28) // max(n2, 1)) // g * g)
                leaves = torch.empty(tchunk * n2, dtype=torch.int32, device=dev)
                out = torch.empty(n2 * width, dtype=torch.float64, device=dev)
                _native.call("ate_forest_predict16", ctypes.addressof(self.params),
                             Xb.data_ptr(), n2, int(oob), self.cap, self.feat.data_ptr(),
                             self.thr.data_ptr(), self.left.data_ptr(), self.val.data_ptr(),
                             self.inbag.data_ptr(), 0 if self.est is None else self.est.data_ptr(),
                             leaves.data_ptr(), tchunk, state.data_ptr(), out.data_ptr(), phases, s)
                if not phases & 4:
                    return None
                if not host:
                    return out.view(n2, width) if width > 1 else out
                res = out.cpu().numpy()
                self.check()
                return res.reshape(n2, width) if width > 1 else res
            if self.packed is None:
                self.packed = torch.zeros(self.params.ntree * self.cap * 2, dtype=torch.int32,
                                          device=dev)
                _native.call("ate_forest_pack", ctypes.addressof(self.params), self.cap,
                             self.feat.data_ptr(), self.thr.data_ptr(), self.left.data_ptr(),
                             self.nnodes.data_ptr(),
                             0 if self.est is None else self.est.data_ptr(),
                             self.packed.data_ptr(), s)
            g = max(1, self.params.group) if self.params.kind == KIND_CAUSAL else 1
            # leaf-index scratch capped at ~1 GiB: trees per chunk, a multiple of the group
            tchunk = max(g, min(self.params.ntree, (1 << 28) // max(n2, 1)) // g * g)
            leaves = torch.empty(tchunk * n2, dtype=torch.int32, device=dev)
            out = torch.empty(n2 * width, dtype=torch.float64, device=dev)
            _native.call("ate_forest_predict", ctypes.addressof(self.params), Xb.data_ptr(), n2,
                         int(oob), self.cap, self.packed.data_ptr(), self.val.data_ptr(),
                         self.inbag.data_ptr(), 0 if self.est is None else self.est.data_ptr(),
                         leaves.data_ptr(), tchunk, state.data_ptr(), out.data_ptr(), phases, s)
            if not phases & 4:
                return None
            if not host:
                return out.view(n2, width) if width > 1 else out
            res = out.cpu().numpy()
        else:
            res = np.empty(n2 * width)
            Xbn = np.ascontiguousarray(Xb.numpy() if isinstance(Xb, torch.Tensor) else Xb)
            lib = _native.cpu()
            fn = lib.atecpu_forest_predict16 if self.exact is not None else \
                lib.atecpu_forest_predict
            rc = fn(
                ctypes.byref(self.params), _ptr(Xbn), ctypes.c_int(n2), ctypes.c_int(int(oob)),
                ctypes.c_int(self.cap), _ptr(self.feat), _ptr(self.thr), _ptr(self.left),
                _ptr(self.val), _ptr(self.inbag), _ptr(self.est) if self.est is not None else None,
                _ptr(state), ctypes.c_int(phases), _ptr(res), ctypes.c_int(_nthreads()))
            if rc != 0:
                raise RuntimeError("atecpu_forest_predict failed")
            if not phases & 4:
                return None
        return res.reshape(n2, width) if width > 1 else res

    def predict_binned(self, Xb, host=True):
        """Predictions for already binned rows (column-major uint8 [p][n2], a device tensor
        for GPU forests, host array/tensor for CPU forests); ``host=False`` keeps a GPU
        forest's predictions on the device."""
        if self.backend == "cpu" and isinstance(Xb, torch.Tensor):
            Xb = Xb.cpu().numpy()
        return self.predict_state(Xb, False, self.new_state(Xb.shape[1]), phases=7, host=host)

    # randomForest-style accessors
    def oob_proba(self):
        return self.predict_raw(None, oob=True)

    def predict_proba(self, X):
        return self.predict_raw(X, oob=False)

    def tree_arrays(self):
        """(feat, thr, left, val, nnodes) as numpy (for parity tests)."""
        self.check()
        f = lambda a: a.cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
        return f(self.feat), f(self.thr), f(self.left), f(self.val), f(self.nnodes)


def _ptr(a):
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.c_void_p)


def fit_forest(X, kind: int, y=None, r1=None, r2=None, ntree=500, mtry=None, min_node=1,
               sampling=0, honesty=False, group=1, mtry_poisson=False, alpha=0.0,
               sample_fraction=0.5, seed=1, backend=None, edges=None, tree_offset=0,
               splits="binned") -> Forest:
    """Grow a forest. X: (n, p) float; kind 0 needs y in {0,1}; kind 1 needs r1 (response);
    kind 2 needs r1 = W~ and r2 = Y~ (centred treatment / outcome).
    ``splits="exact"``: randomForest split semantics (every distinct value a candidate,
    midpoint thresholds); ``edges`` is then an ExactBins (default: from X)."""
    X = np.asarray(X.detach().cpu().numpy() if isinstance(X, torch.Tensor) else X, dtype=np.float64)
    if backend is None:
        backend = "gpu" if torch.cuda.is_available() else "cpu"
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "gpu" else None
    if splits == "exact":
        eb = edges if isinstance(edges, ExactBins) else exact_bins(X)
        Xb = torch.from_numpy(eb.bin(X))          # training rows: ranks either way
        if dev is not None:
            Xb = Xb.to(dev)
        return fit_forest_exact(Xb, eb, kind, y=y, r1=r1, r2=r2, ntree=ntree, mtry=mtry,
                                min_node=min_node, sampling=sampling, honesty=honesty,
                                group=group, mtry_poisson=mtry_poisson, alpha=alpha,
                                sample_fraction=sample_fraction, seed=seed,
                                tree_offset=tree_offset)
    if splits != "binned":
        raise ValueError(f"splits must be 'binned' or 'exact', got {splits!r}")
    Xsrc = X
    if edges is None:
        if dev is not None and X.size >= DEVICE_EDGES_MIN:
            # large inputs: sort on the device (same edges bit for bit), bin from there
            Xsrc = torch.as_tensor(X, device=dev)
            edges, ne = bin_edges_device(Xsrc)
        else:
            edges, ne = bin_edges(X)
    else:
        edges, ne = edges
    Xb = bin_matrix(Xsrc, edges, ne, dev)
    del Xsrc
    return fit_forest_binned(Xb, (edges, ne), kind, y=y, r1=r1, r2=r2, ntree=ntree, mtry=mtry,
                             min_node=min_node, sampling=sampling, honesty=honesty, group=group,
                             mtry_poisson=mtry_poisson, alpha=alpha,
                             sample_fraction=sample_fraction, seed=seed, tree_offset=tree_offset)


LEVEL_MIN_ROWS = 1 << 17     # training rows from which the level engine grows a forest


def use_level_engine(fp: ForestParams) -> bool:
    """ATE_FOREST_ENGINE = "tree" (one workgroup per tree), "level" (GPU-wide level
    steps; randomForest sampling only) or "auto" (level for >= LEVEL_MIN_ROWS rows)."""
    from . import forest_level as LV
    mode = os.environ.get("ATE_FOREST_ENGINE", "auto")
    if mode == "tree" or not LV.supported(fp):
        return False
    return mode == "level" or fp.n >= LEVEL_MIN_ROWS


def fit_forest_binned(Xb, edges, kind: int, y=None, r1=None, r2=None, ntree=500, mtry=None,
                      min_node=1, sampling=0, honesty=False, group=1, mtry_poisson=False,
                      alpha=0.0, sample_fraction=0.5, seed=1, tree_offset=0) -> Forest:
    """``fit_forest`` on an already binned column-major uint8 matrix ``Xb`` [p][n]: a device
    tensor grows on the GPU (csrc/forest.hip), a host array on the CPU engine; both grow the
    same trees. ``edges`` = (edges, nedges) the bins came from. y / r1 / r2 may be device
    tensors (no host round trip of the responses for HBM-resident panels)."""
    edges, ne = edges
    gpu = isinstance(Xb, torch.Tensor) and Xb.is_cuda
    p, n = Xb.shape
    if mtry is None:
        mtry = max(1, int(math.floor(math.sqrt(p))))
    fp = ForestParams(kind=kind, sampling=sampling, ntree=ntree, mtry=min(mtry, p),
                      min_node=min_node, honesty=int(honesty), group=max(1, group),
                      mtry_poisson=int(mtry_poisson), alpha=alpha,
                      sample_fraction=sample_fraction, pois0=math.exp(-min(mtry, p)),
                      seed=seed, p=p, n=n, t0=tree_offset)
    cap = 2 * n + 1
    need_est = sampling == 1
    if gpu:
        dev = Xb.device

        def t(a, dt, fix=False):
            if a is None:
                return None
            if isinstance(a, torch.Tensor):
                a = a.to(dev)
                if fix:   # 2^-32 fixed point, round half away from zero (to_fix)
                    v = a.double() * FIX
                    return torch.where(v >= 0, torch.floor(v + 0.5), torch.ceil(v - 0.5)).to(dt)
                return a.to(dt)
            return torch.as_tensor(to_fix(a) if fix else np.asarray(a), device=dev, dtype=dt)

        yt = t(y, torch.uint8)
        r1t, r2t = t(r1, torch.int64, True), t(r2, torch.int64, True)
        Xb = Xb.contiguous()
        if use_level_engine(fp):
            # large training sets: all trees grown together, level by level, across the
            # whole GPU (csrc/forest_level.hip); same trees as the per-tree kernel
            from . import forest_level as LV
            cap, feat, thr, left, val, nnodes, inbag = LV.grow(Xb, fp, yt, r1t)
            return Forest(fp, "gpu", cap, feat, thr, left, val, nnodes, inbag, None, edges, ne,
                          Xb)
        feat = torch.empty(ntree * cap, dtype=torch.int32, device=dev)
        thr = torch.empty_like(feat)
        left = torch.empty_like(feat)
        val = torch.zeros(ntree * cap, dtype=torch.float64, device=dev)
        nnodes = torch.empty(ntree, dtype=torch.int32, device=dev)
        inbag = torch.empty(ntree * n, dtype=torch.uint8, device=dev)
        est = torch.zeros(ntree * cap * 5, dtype=torch.int64, device=dev) if need_est else None
        sb = _native.hip().ate_forest_scratch_bytes(n, ntree)
        scratch = torch.empty(sb, dtype=torch.uint8, device=dev)
        p_ = lambda a: 0 if a is None else a.data_ptr()
        _native.call("ate_forest_fit", ctypes.addressof(fp), Xb.data_ptr(), p_(yt), p_(r1t),
                     p_(r2t), cap, feat.data_ptr(), thr.data_ptr(), left.data_ptr(),
                     val.data_ptr(), nnodes.data_ptr(), inbag.data_ptr(), p_(est),
                     scratch.data_ptr(), int(os.environ.get("ATE_FOREST_NW", "0")),
                     torch.cuda.current_stream().cuda_stream)
        del scratch
        return Forest(fp, "gpu", cap, feat, thr, left, val, nnodes, inbag, est, edges, ne, Xb)
    h = lambda a: None if a is None else (a.cpu().numpy() if isinstance(a, torch.Tensor) else
                                           np.asarray(a))
    Xbn = np.ascontiguousarray(h(Xb), dtype=np.uint8)
    ycls = None if y is None else h(y).astype(np.uint8)
    r1f = None if r1 is None else to_fix(h(r1))
    r2f = None if r2 is None else to_fix(h(r2))
    feat = np.empty(ntree * cap, dtype=np.int32)
    thr = np.empty_like(feat)
    left = np.empty_like(feat)
    val = np.zeros(ntree * cap)
    nnodes = np.empty(ntree, dtype=np.int32)
    inbag = np.empty(ntree * n, dtype=np.uint8)
    est = np.zeros(ntree * cap * 5, dtype=np.int64) if need_est else None
    lib = _native.cpu()
    rc = lib.atecpu_forest_fit(ctypes.byref(fp), _ptr(Xbn), _ptr(ycls), _ptr(r1f), _ptr(r2f),
                               ctypes.c_int(cap), _ptr(feat), _ptr(thr), _ptr(left), _ptr(val),
                               _ptr(nnodes), _ptr(inbag), _ptr(est), ctypes.c_int(_nthreads()))
    if rc != 0:
        raise RuntimeError("atecpu_forest_fit failed")
    return Forest(fp, "cpu", cap, feat, thr, left, val, nnodes, inbag, est, edges, ne, Xbn)


def exact_row_order(Xb: torch.Tensor) -> torch.Tensor:
    """[p][n] uint32 entries (value rank << 16 | row) per feature in ascending order (held in
    an int32 tensor): the forest-wide value order every tree filters to its in-bag rows
    (csrc/forest_exact.hip). Ties are in row order; the splits do not depend on it."""
    p, n = Xb.shape
    key = (Xb.to(torch.int64) << 16) | torch.arange(n, device=Xb.device, dtype=torch.int64)
    key = torch.sort(key, dim=1).values
    return torch.where(key >= 2 ** 31, key - 2 ** 32, key).to(torch.int32).contiguous()


def exact_mcap(n: int, sampling: int, group: int, sample_fraction: float, honesty: bool) -> int:
    """A tree's in-bag (J1) row count as the exact-split kernel's sampling draws it (the bound
    its per-position scratch is sized by): randomForest bootstrap -> n (distinct rows <= n);
    grf: the group's half-sample floor(n / 2) (group > 1), the tree's subsample of it
    floor(nh * min(1, sample_fraction * group)), or floor(n * sample_fraction) (group 1), then
    honesty's half (ns // 2)."""
    if sampling == 0:
        return n
    if group > 1:
        nh = n // 2
        f = min(1.0, sample_fraction * group)
        ns = nh if f >= 1.0 else int(math.floor(nh * f))
    else:
        ns = int(math.floor(n * sample_fraction))
    return max(1, ns // 2 if honesty else ns)


def fit_forest_exact(Xb, eb, kind: int, y=None, r1=None, r2=None, ntree=500, mtry=None,
                     min_node=1, sampling=0, honesty=False, group=1, mtry_poisson=False,
                     alpha=0.0, sample_fraction=0.5, seed=1, tree_offset=0) -> Forest:
    """Exact-split forest on value-rank bins ``Xb`` (uint16 [p][n]; a device tensor grows on
    the GPU, csrc/forest_exact.hip, a host one on the CPU twin). randomForest sampling
    (``sampling=0``): kinds 0/1, midpoint thresholds. grf sampling (``sampling=1``): kinds
    1/2 with half-samples / little bags (``group``), ``honesty`` and the J2 estimation
    statistics; the left value is the threshold. ``eb``: ExactBins (or, on the GPU, its
    DeviceExactBins)."""
    if sampling == 0 and kind not in (KIND_CLASS, KIND_REG):
        raise ValueError("exact-split randomForest forests: classification or regression")
    if sampling == 1 and kind not in (KIND_REG, KIND_CAUSAL):
        raise ValueError("exact-split grf forests: regression or causal")
    if kind == KIND_CAUSAL and r2 is None:
        raise ValueError("causal forests need r1 = W~ and r2 = Y~")
    gpu = isinstance(Xb, torch.Tensor) and Xb.is_cuda
    p, n = Xb.shape
    if n > EXACT_MAX_ROWS:
        raise ValueError(f"exact-split forests take at most {EXACT_MAX_ROWS} rows (got {n})")
    if mtry is None:
        mtry = max(1, int(math.floor(math.sqrt(p))))
    fp = ForestParams(kind=kind, sampling=sampling, ntree=ntree, mtry=min(mtry, p),
                      min_node=min_node, honesty=int(honesty), group=max(1, group),
                      mtry_poisson=int(mtry_poisson), alpha=alpha,
                      sample_fraction=sample_fraction, pois0=math.exp(-min(mtry, p)), seed=seed,
                      p=p, n=n, t0=tree_offset)
    cap = 2 * n + 1
    need_est = sampling == 1
    h = lambda a: None if a is None else (a.cpu().numpy() if isinstance(a, torch.Tensor) else
                                           np.asarray(a))
    if gpu:
        dev = Xb.device
        # device responses stay on the device (capturable estimator bodies)
        if isinstance(y, torch.Tensor):
            yt = y.to(dev, torch.uint8)
        else:
            yt = None if y is None else torch.as_tensor(h(y).astype(np.uint8), device=dev)

        def fixt(r):
            if r is None:
                return None
            if isinstance(r, torch.Tensor):
                v = r.to(dev, torch.float64) * FIX
                return torch.where(v >= 0, torch.floor(v + 0.5), torch.ceil(v - 0.5)).to(torch.int64)
            return torch.as_tensor(to_fix(h(r)), device=dev)
        r1t, r2t = fixt(r1), fixt(r2)
        de = eb.on(dev) if isinstance(eb, ExactBins) else eb
        vals, nval = de.vals, de.nval
        feat = torch.empty(ntree * cap, dtype=torch.int32, device=dev)
        thr = torch.empty_like(feat)
        left = torch.empty_like(feat)
        val = torch.zeros(ntree * cap, dtype=torch.float64, device=dev)
        nnodes = torch.empty(ntree, dtype=torch.int32, device=dev)
        inbag = torch.empty(ntree * n, dtype=torch.uint8, device=dev)
        est = torch.zeros(ntree * cap * 5, dtype=torch.int64, device=dev) if need_est else None
        mc = exact_mcap(n, sampling, max(1, group), sample_fraction, bool(honesty))
        per = _native.hip().ate_forest_exact_scratch_bytes(n, p, mc, 1)
        if per > 4 * EXACT_AUTO_LIST_BYTES:
            import warnings
            warnings.warn(f"exact-split forest with p = {p}, {mc} in-bag rows: {per >> 20} MB "
                          "of scratch per tree, few trees per launch; splits='binned' (or "
                          "'auto') suits wide panels", RuntimeWarning, stacklevel=3)
        # trees per launch: two resident per CU, so a launch wants >= 512 of them and as
        # few tails as possible. A 1-GiB scratch cap held 264 trees of 5e4 rows (half the CUs
        # idle, a tail per launch; config 4 2.53 s); when 1 GiB cannot hold the whole forest
        # the cap is 2048 trees' worth up to 8 GiB (config 4 1.43 s, same trees;
        # profiles/r04_cfg4). ATE_EXACT_SCRATCH_MB overrides.
        # Inside a stream capture (estimator graphs) the scratch would live as long as the
        # graph's private pool: capped at 1 GiB there, so cached graphs do not each pin GBs.
        env_mb = int(os.environ.get("ATE_EXACT_SCRATCH_MB", "0"))
        capturing = torch.cuda.is_current_stream_capturing()
        cap_b = env_mb << 20 if env_mb else \
            (1 << 30 if capturing or (1 << 30) // per >= ntree else min(8 << 30, 2048 * per))
        chunk = max(1, min(ntree, cap_b // per))
        scratch = torch.empty(per * chunk, dtype=torch.uint8, device=dev)
        Xb = Xb.contiguous()
        # the forest's rows in value order per feature (a stable sort of the ranks, once per
        # forest): every tree's large nodes read these lists filtered to their rows instead
        # of sorting per node (csrc/forest_exact.hip)
        order = exact_row_order(Xb)
        p_ = lambda a: 0 if a is None else a.data_ptr()
        s = torch.cuda.current_stream().cuda_stream
        for t0 in range(0, ntree, chunk):
            _native.call("ate_forest_fit_exact", ctypes.addressof(fp), t0, min(chunk, ntree - t0),
                         mc, Xb.data_ptr(), order.data_ptr(), vals.data_ptr(), de.ldv, nval.data_ptr(), p_(yt), p_(r1t),
                         p_(r2t), cap, feat.data_ptr(), thr.data_ptr(), left.data_ptr(),
                         val.data_ptr(), nnodes.data_ptr(), inbag.data_ptr(), p_(est),
                         scratch.data_ptr(), s)
        del scratch
        # a tree whose in-bag count exceeded the host's bound mc returns nnodes = -1: an empty
        # tree must not pass silently. The count stays on the device and Forest.check() reads
        # it at the first host read (a host sync here made the next fit's host-side set-up
        # wait for this fit: config 4 0.71 -> 0.78-0.82 s). Inside a graph capture the check
        # runs on the eager first call of the estimator instead.
        ovf = None if torch.cuda.is_current_stream_capturing() else \
            ((nnodes < 0).sum(), ntree, mc)
        return Forest(fp, "gpu", cap, feat, thr, left, val, nnodes, inbag, est, None, None, Xb,
                      exact=eb, overflow=ovf)
    Xbn = np.ascontiguousarray(h(Xb), dtype=np.uint16)
    ycls = None if y is None else h(y).astype(np.uint8)
    r1f = None if r1 is None else to_fix(h(r1))
    r2f = None if r2 is None else to_fix(h(r2))
    feat = np.empty(ntree * cap, dtype=np.int32)
    thr = np.empty_like(feat)
    left = np.empty_like(feat)
    val = np.zeros(ntree * cap)
    nnodes = np.empty(ntree, dtype=np.int32)
    inbag = np.empty(ntree * n, dtype=np.uint8)
    est = np.zeros(ntree * cap * 5, dtype=np.int64) if need_est else None
    vals = np.ascontiguousarray(eb.vals)
    nval = np.ascontiguousarray(eb.nval, dtype=np.int32)
    rc = _native.cpu().atecpu_forest_fit_exact(
        ctypes.byref(fp), _ptr(Xbn), _ptr(vals), ctypes.c_int(eb.ldv), _ptr(nval), _ptr(ycls),
        _ptr(r1f), _ptr(r2f), ctypes.c_int(cap), _ptr(feat), _ptr(thr), _ptr(left), _ptr(val),
        _ptr(nnodes), _ptr(inbag), _ptr(est), ctypes.c_int(_nthreads()))
    if rc != 0:
        raise RuntimeError("atecpu_forest_fit_exact failed")
    return Forest(fp, "cpu", cap, feat, thr, left, val, nnodes, inbag, est, None, None, Xbn,
                  exact=eb)


# ------------------------------------------------------------------ public learners
def rf_classifier(X, y, num_trees=500, mtry=None, nodesize=1, seed=1, backend=None,
                  splits="binned") -> Forest:
    """randomForest(factor(y) ~ X, ntree, type="classification") (ate_functions.R:169).
    ``splits="exact"``: randomForest's split semantics on continuous covariates."""
    return fit_forest(X, KIND_CLASS, y=y, ntree=num_trees, mtry=mtry, min_node=nodesize,
                      seed=seed, backend=backend, splits=splits)


def rf_regressor(X, y, num_trees=500, mtry=None, nodesize=5, seed=1, backend=None,
                 splits="binned") -> Forest:
    """Breiman regression forest (bootstrap, variance-reduction splits)."""
    p = np.asarray(X).shape[1]
    return fit_forest(X, KIND_REG, r1=y, ntree=num_trees, mtry=mtry or max(1, p // 3),
                      min_node=nodesize, seed=seed, backend=backend, splits=splits)


def grf_mtry(p):
    return min(int(math.ceil(math.sqrt(p) + 20)), p)


def regression_forest(X, y, num_trees=2000, honesty=True, min_node=5, alpha=0.05,
                      sample_fraction=0.5, group=2, seed=1, backend=None, splits="binned",
                      edges=None) -> Forest:
    """grf::regression_forest defaults; OOB predictions via ``oob_predict``.
    ``splits``: "exact" (grf's exact values), "binned" or "auto" (exact up to 65,536 rows)."""
    X = np.asarray(X, dtype=np.float64)
    p = X.shape[1]
    return fit_forest(X, KIND_REG, r1=y, ntree=num_trees, mtry=grf_mtry(p), min_node=min_node,
                      sampling=1, honesty=honesty, group=group, mtry_poisson=True, alpha=alpha,
                      sample_fraction=sample_fraction, seed=seed, backend=backend,
                      splits=resolve_splits(splits, X.shape[0], X.shape[1]), edges=edges)


@dataclass
class CausalForestFit:
    forest: Forest
    y_hat: np.ndarray
    w_hat: np.ndarray
    tau_oob: np.ndarray
    var_oob: np.ndarray
    Y: np.ndarray
    W: np.ndarray


def causal_forest(X, Y, W, num_trees=2000, honesty=True, min_node=5, alpha=0.05,
                  sample_fraction=0.5, group=2, seed=12345, nuisance_trees=None,
                  backend=None, comm=None, splits="auto", nuisance_group=1) -> CausalForestFit:
    """grf::causal_forest(X, Y, W, num.trees, honesty=TRUE, seed) (ate_replication.Rmd:250-255):
    OOB regression forests for Y.hat and W.hat (grf's orthogonalisation forests:
    max(50, num.trees / 4) trees, ``ci.group.size = 1`` -> ``nuisance_group``), then causal
    trees in little bags of ``group`` on the centred (W - W.hat, Y - Y.hat). ``splits``:
    "auto" = grf's exact split values up to 65,536 rows (the tutorial), 256-bin histograms
    above; "exact" / "binned" force one."""
    X = np.asarray(X, dtype=np.float64)
    Y = np.asarray(Y, dtype=np.float64)
    W = np.asarray(W, dtype=np.float64)
    nt = nuisance_trees or max(50, num_trees // 4)
    splits = resolve_splits(splits, X.shape[0], X.shape[1])
    edges = exact_bins(X) if splits == "exact" else bin_edges(X)
    p = X.shape[1]
    grf = dict(mtry=grf_mtry(p), min_node=min_node, sampling=1, honesty=honesty,
               mtry_poisson=True, alpha=alpha, sample_fraction=sample_fraction, backend=backend,
               edges=edges, splits=splits)
    if comm is not None and comm.world_size > 1:
        # tree-parallel: every rank grows its share of each forest (C05 all-reduces)
        fy = fit_forest_sharded(X, KIND_REG, nt, comm, r1=Y, seed=seed + 1, group=nuisance_group,
                                **grf)
        fw = fit_forest_sharded(X, KIND_REG, nt, comm, r1=W, seed=seed + 2, group=nuisance_group,
                                **grf)
        y_hat = predict_tree_parallel(fy, comm, oob=True)
        w_hat = predict_tree_parallel(fw, comm, oob=True)
        y_hat = np.where(np.isnan(y_hat), Y.mean(), y_hat)
        w_hat = np.where(np.isnan(w_hat), W.mean(), w_hat)
        fc = fit_forest_sharded(X, KIND_CAUSAL, num_trees, comm, r1=W - w_hat, r2=Y - y_hat,
                                seed=seed, group=group, **grf)
        out = predict_tree_parallel(fc, comm, oob=True)
        return CausalForestFit(fc, y_hat, w_hat, out[:, 0], out[:, 1], Y, W)
    fy = fit_forest(X, KIND_REG, r1=Y, ntree=nt, seed=seed + 1, group=nuisance_group, **grf)
    fw = fit_forest(X, KIND_REG, r1=W, ntree=nt, seed=seed + 2, group=nuisance_group, **grf)
    y_hat = fy.predict_raw(None, oob=True)
    w_hat = fw.predict_raw(None, oob=True)
    y_hat = np.where(np.isnan(y_hat), Y.mean(), y_hat)
    w_hat = np.where(np.isnan(w_hat), W.mean(), w_hat)
    fc = fit_forest(X, KIND_CAUSAL, r1=W - w_hat, r2=Y - y_hat, ntree=num_trees, seed=seed,
                    group=group, **grf)
    out = fc.predict_raw(None, oob=True)
    return CausalForestFit(fc, y_hat, w_hat, out[:, 0], out[:, 1], Y, W)


AIPW_TEXTBOOK_CLIP = 1e-6    # compat="textbook": W.hat clipped to [clip, 1 - clip]


def overlap_warning(w_min: float, w_max: float, what="W.hat"):
    """grf does not clip the propensity in its AIPW average effect; it warns when the
    estimated propensities come close to 0 or 1 (poor overlap). Same here: a warning, and
    with W.hat exactly 0 or 1 the scores are infinite (as in grf)."""
    if not (w_min > 0.05 and w_max < 0.95):
        import warnings
        warnings.warn(f"estimated propensities {what} span [{w_min:.3g}, {w_max:.3g}]: poor "
                      "overlap, the AIPW average effect may be unstable (grf's warning; "
                      "compat='textbook' clips W.hat)", RuntimeWarning, stacklevel=3)


def average_treatment_effect(cf: CausalForestFit, clip: float | None = None):
    """grf ``estimate_average_effect`` / ``average_treatment_effect`` (AIPW):
    Gamma_i = tau_i + (W_i - W.hat_i)/(W.hat_i (1 - W.hat_i)) * (Y~_i - tau_i W~_i);
    estimate = mean(Gamma), std.err = sd(Gamma)/sqrt(n). grf does not clip W.hat (it warns
    on poor overlap): ``clip`` = None reproduces that; a float clips W.hat to
    [clip, 1 - clip] (the compat="textbook" option of the estimators)."""
    w_res = cf.W - cf.w_hat
    y_res = cf.Y - cf.y_hat
    tau = np.where(np.isnan(cf.tau_oob), np.nanmean(cf.tau_oob), cf.tau_oob)
    overlap_warning(float(np.min(cf.w_hat)), float(np.max(cf.w_hat)))
    what = cf.w_hat if clip is None else np.clip(cf.w_hat, clip, 1 - clip)
    gamma = tau + w_res / (what * (1 - what)) * (y_res - tau * w_res)
    n = len(gamma)
    return float(gamma.mean()), float(gamma.std(ddof=1) / math.sqrt(n))


# ------------------------------------------------------------------ tree parallelism (C05)
def tree_shard(ntree: int, group: int, rank: int, world: int):
    """(first tree, tree count) of this rank; shards are whole little-bag groups."""
    from ..parallel.dist import shard_range
    g = max(1, group)
    g0, ng = shard_range(-(-ntree // g), rank, world)
    t0 = g0 * g
    return t0, max(0, min(ntree, (g0 + ng) * g) - t0)


def fit_forest_sharded(X, kind, ntree, comm, group=1, **kw) -> Forest:
    """Every rank holds all rows (binned panel replicated) and grows its share of the
    trees; tree t uses the same Philox streams as on a single device (global id)."""
    t0, cnt = tree_shard(ntree, group, comm.rank, comm.world_size)
    if cnt < 1:
        raise ValueError(f"{ntree} trees cannot be sharded over {comm.world_size} ranks "
                         f"in groups of {group}")
    return fit_forest(X, kind, ntree=max(cnt, 0), group=group, tree_offset=t0, **kw)


def predict_tree_parallel(forest: Forest, comm, X=None, oob=False, Xb=None, host=True):
    """Forest prediction with trees sharded over ranks: all-reduce the per-tree sums
    (C05), then (causal forests) the little-bag group sums, then finalise locally. The
    sums are int64 fixed point (``Forest.new_state``): every world size gives the same
    bits as one device growing all the trees.
    ``Xb``: already binned rows (column-major uint8 [p][n2]) instead of ``X``.
    ``host=False`` (GPU forests): the predictions stay a device tensor."""
    if Xb is None:
        Xb = forest._bins(X)
    n2 = Xb.shape[1]
    st = forest.new_state(n2)
    t = st if isinstance(st, torch.Tensor) else torch.from_numpy(st)
    forest.predict_state(Xb, oob, st, phases=1)
    k = 5 if forest.params.kind == KIND_CAUSAL else 2
    if comm.world_size > 1:
        comm.all_reduce_(t[:k * n2])
    if forest.params.kind == KIND_CAUSAL:
        forest.predict_state(Xb, oob, st, phases=2)
        if comm.world_size > 1:
            comm.all_reduce_(t[5 * n2:])
    return forest.predict_state(Xb, oob, st, phases=4, host=host)
