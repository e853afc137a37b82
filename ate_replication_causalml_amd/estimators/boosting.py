"""DML-PLR with histogram-GBDT nuisances (BASELINE config 5: "N=1e8 p=2000 DML with
histogram-GBDT nuisance, full panel resident in 8x288 GB HBM").

For each of K folds, E[Y|X] and E[W|X] are boosted on the other folds (``train``
mask over the resident binned panel — no row copies) and predicted on fold k; the
held-out residuals feed the Neyman-orthogonal PLR score (same moments/finalisation
as the LASSO cross-fit, ops/stats.py). ``dist`` shards rows across ranks: histograms
(C04) and score moments (C06) are all-reduced, CV folds use global fold ids.
"""
from __future__ import annotations

import numpy as np
import torch

from ..models import gbdt as G
from ..ops import stats as S
from ..parallel import rng
from .common import as_np, read_result, resolve_device


def _loss(v):
    return "logistic" if bool(np.all((v == 0) | (v == 1))) else "squared"


def dml_plr_gbdt(Y, W, X, folds=5, n_trees=100, depth=6, lr=0.1, lam=1.0, min_child=1.0,
                 seed=1991, fold_stream=0, method="DML cross-fit (GBDT)", device=None,
                 dist=None):
    dev = resolve_device(device)
    Yn, Wn, Xn = as_np(Y), as_np(W), as_np(X)
    n = len(Yn)
    fid = dist.fold_ids(folds, seed, fold_stream) if dist is not None else \
        rng.fold_ids(n, folds, seed, fold_stream)
    backend = "gpu" if dev.type == "cuda" else "cpu"
    edges = G.global_bin_edges(Xn, dist, device=dev)
    Xb = G.binned(Xn, edges, dev)          # binned once, shared by all 2K fits
    ey = np.empty(n)
    ew = np.empty(n)
    kw = dict(n_trees=n_trees, depth=depth, lr=lr, lam=lam, min_child=min_child,
              backend=backend, edges=edges, dist=dist, Xb=Xb)

    def response(m):
        f = m.scores.cpu().numpy() if isinstance(m.scores, torch.Tensor) else m.scores
        return 1.0 / (1.0 + np.exp(-f)) if m.loss == "logistic" else f

    for k in range(folds):
        ho = fid == k
        # held-out predictions = the trainer's running scores of the rows it skipped
        ey[ho] = response(G.fit_gbdt(None, Yn, loss=_loss(Yn), train=~ho, **kw))[ho]
        ew[ho] = response(G.fit_gbdt(None, Wn, loss=_loss(Wn), train=~ho, **kw))[ho]
    yr = torch.as_tensor(Yn - ey, device=dev)
    wr = torch.as_tensor(Wn - ew, device=dev)
    mom = S.dml_moments(yr, wr).clone()
    if dist is not None:
        dist.sum_(mom)
    res = S.dml_finalize(mom, "plr")
    return read_result(res, method, n=dist.n_total if dist is not None else n)


def bin_panel(pan, edges=None, edge_rows=200_000):
    """Row-major uint8 bins [n_real][ldr] of the panel's feature columns, binned on the
    device (csrc/gbdt.hip gbdt_bin_panel_kernel; no host copy of X). Edges default to
    quantile edges of an evenly strided device sample of the real rows.
    Returns (Xr, ldr, edges, rows) with ``rows`` the panel row of each compact row."""
    from .. import _native
    from ..models import forest as F
    dev = pan.device
    X = pan.data
    p = len(pan.xcols)
    r0 = np.asarray(pan.seg_bounds[:, 0], dtype=np.int64)
    nr = np.asarray(pan.seg_nreal, dtype=np.int64)
    c0 = np.concatenate([[0], np.cumsum(nr)[:-1]]).astype(np.int64)
    n = int(nr.sum())
    rows = torch.cat([torch.arange(int(a), int(a + m), device=dev) for a, m in zip(r0, nr)])
    if edges is None:
        xc = torch.as_tensor(pan.xcols, dtype=torch.long, device=dev)
        pick = torch.as_tensor(np.linspace(0, n - 1, num=min(n, edge_rows)).astype(np.int64),
                               device=dev)
        edges = F.bin_edges_device(X.index_select(0, xc).index_select(1, rows[pick]).t().double())
    ldr = -(-p // 32) * 32
    Xr = torch.zeros((n, ldr), dtype=torch.uint8, device=dev)
    code = {torch.bfloat16: 0, torch.float32: 1}[X.dtype]
    t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)
    e, ne = t(edges[0], torch.float64), t(edges[1], torch.int32)
    xci = t(np.asarray(pan.xcols), torch.int32)
    r0t, nrt, c0t = t(r0, torch.int64), t(nr, torch.int64), t(c0, torch.int64)
    _native.call("ate_gbdt_bin_panel", X.data_ptr(), code, pan.cm_ld, xci.data_ptr(), p,
                 r0t.data_ptr(), nrt.data_ptr(), c0t.data_ptr(), pan.nseg, n, e.data_ptr(),
                 ne.data_ptr(), Xr.data_ptr(), ldr, torch.cuda.current_stream().cuda_stream)
    return Xr, ldr, edges, rows


def dml_plr_gbdt_panel(pan, n_trees=100, depth=6, lr=0.1, lam=1.0, min_child=1.0,
                       method="DML cross-fit (GBDT)"):
    """Config 5 on an HBM-resident panel (data/device_dgp.synthetic_panel, segment k =
    fold k): device binning (``bin_panel``), then the same K-fold cross-fit as
    ``dml_plr_gbdt`` on the resident row-major bins."""
    dev = pan.device
    Xr, ldr, edges, rows = bin_panel(pan)
    K = pan.nseg
    nr = np.asarray(pan.seg_nreal, dtype=np.int64)
    n = int(nr.sum())
    Yn = pan.col("Y").index_select(0, rows).double().cpu().numpy()
    Wn = pan.col("W").index_select(0, rows).double().cpu().numpy()
    fid = np.repeat(np.arange(K), nr)
    kw = dict(n_trees=n_trees, depth=depth, lr=lr, lam=lam, min_child=min_child,
              backend="gpu", edges=edges, Xb=(Xr, ldr))

    def response(m):
        f = m.scores.cpu().numpy() if isinstance(m.scores, torch.Tensor) else m.scores
        return 1.0 / (1.0 + np.exp(-f)) if m.loss == "logistic" else f

    ey = np.empty(n)
    ew = np.empty(n)
    for k in range(K):
        ho = fid == k
        ey[ho] = response(G.fit_gbdt(None, Yn, loss=_loss(Yn), train=~ho, **kw))[ho]
        ew[ho] = response(G.fit_gbdt(None, Wn, loss=_loss(Wn), train=~ho, **kw))[ho]
    mom = S.dml_moments(torch.as_tensor(Yn - ey, device=dev),
                        torch.as_tensor(Wn - ew, device=dev)).clone()
    return read_result(S.dml_finalize(mom, "plr"), method, n=n)
