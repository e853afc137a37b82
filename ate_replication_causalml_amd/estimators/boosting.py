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
