"""Device forest estimators: E8 doubly robust with RF propensity, E12/E13 the
reference's two-half "double ML" with RF learners, E15 causal forest (grf) ATE.

Forests grow on the GPU (csrc/forest.hip) when a GPU is present; ``backend="cpu"``
runs the host C++ twin (bit-identical trees). Nuisance GLMs and score reductions use
the device kernels of estimators/linear.py.
"""
from __future__ import annotations

import numpy as np
import torch

from ..models import forest as F
from ..reference import estimators as R
from ..result import AteResult
from . import linear as D
from .common import as_np, resolve_device


def _backend(device):
    dev = resolve_device(device)
    return "gpu" if dev.type == "cuda" else "cpu"


def _rf_oob(Xn, y, num_trees, seed, dev, comm):
    if comm is not None and comm.world_size > 1:
        fr = F.fit_forest_sharded(Xn, F.KIND_CLASS, num_trees, comm, y=y, seed=seed,
                                  backend=_backend(dev))
        return F.predict_tree_parallel(fr, comm, oob=True)
    return F.rf_classifier(Xn, y, num_trees=num_trees, seed=seed, backend=_backend(dev)).oob_proba()


def aipw_rf(Y, W, X, num_trees=100, bootstrap_se=False, B=1000, seed=1991, forest_seed=12325,
            compat="reference", method="Doubly Robust with Random Forest PS", device=None,
            dtype="f64", comm=None, graph=True):
    """E8 ``doubly_robust`` (ate_functions.R:149-207): logistic outcome model (with the
    mutate_ quirk Q6 under compat="reference"), randomForest OOB propensity clipped (Q9).
    ``comm``: tree-parallel propensity forest over ranks (rows replicated, C05)."""
    dev = resolve_device(device)
    Yn, Wn, Xn = as_np(Y), as_np(W), as_np(X)
    if graph and (comm is None or comm.world_size == 1) and dev.type == "cuda":
        # one hipGraph launch: outcome IRLS + counterfactual predictions, the propensity
        # forest (growth, OOB votes, clipping) and the AIPW score, over the binned matrix
        # (bin edges come from the data, so binning stays in front of the graph)
        from ..utils.graphs import estimator_graphs
        po = D._outcome_panel(Yn, Wn, Xn, dtype, dev)
        edges = F.bin_edges(Xn)
        Xb = F.bin_matrix(Xn, *edges, dev)
        y = torch.as_tensor(Yn, device=dev)
        w = torch.as_tensor(Wn, device=dev)
        out, g = estimator_graphs.run("aipw_rf", _aipw_rf_body, (po, Xb, y, w), num_trees,
                                      forest_seed, compat, bootstrap_se, B, seed)
        v = out.cpu().numpy()
        return AteResult.make(method, v[0], v[1], n_oob_nan=int(v[2]), hipgraph=g)
    mu0, mu1 = D.outcome_mu(Yn, Wn, Xn, counterfactual_quirk=(compat == "reference"),
                            device=dev, dtype=dtype)
    p_raw = _rf_oob(Xn, Wn, num_trees, forest_seed, dev, comm)
    p = torch.as_tensor(p_raw, device=dev)
    from ..ops import stats as S
    S.clip_propensity_(p)
    return D.aipw_from_nuisances(method, Yn, Wn, p, mu0, mu1, bootstrap_se, B, seed, compat, dev,
                                 n_oob_nan=int(np.isnan(p_raw).sum()))


def _aipw_rf_body(po, Xb, y, w, num_trees, forest_seed, compat, bootstrap_se, B, seed):
    """Device body of aipw_rf (no host sync): [ate, se, #OOB-NaN propensities]."""
    from ..ops import stats as S
    mu0, mu1 = D._outcome_fit(po, compat == "reference")
    fr = F.fit_forest_binned(Xb, (None, None), F.KIND_CLASS, y=w, ntree=num_trees,
                             seed=forest_seed)
    p = fr.predict_state(Xb, True, fr.new_state(Xb.shape[1]), 7, host=False).clone()
    nan = torch.isnan(p).sum().double().reshape(1)
    S.clip_propensity_(p)
    res = D._aipw_core(y, w, p, mu0, mu1, bootstrap_se, B, seed, compat)
    return torch.cat([res, nan])


def chernozhukov(Y, W, X, idx1, idx2, num_trees, seed=123, device=None, comm=None):
    """One half of ``double_ml`` (ate_functions.R:332-369): RF classifier for W on idx1,
    for Y on idx2, both predicted on all rows (in-sample for the training half, Q14)."""
    be = _backend(device)
    Yn, Wn, Xn = as_np(Y), as_np(W), as_np(X)
    edges = F.bin_edges(Xn)
    if comm is not None and comm.world_size > 1:
        rf1 = F.fit_forest_sharded(Xn[idx1], F.KIND_CLASS, num_trees, comm, y=Wn[idx1], seed=seed,
                                   backend=be, edges=edges)
        rf2 = F.fit_forest_sharded(Xn[idx2], F.KIND_CLASS, num_trees, comm, y=Yn[idx2],
                                   seed=seed + 1, backend=be, edges=edges)
        ew = F.predict_tree_parallel(rf1, comm, X=Xn)
        ey = F.predict_tree_parallel(rf2, comm, X=Xn)
    else:
        rf1 = F.fit_forest(Xn[idx1], F.KIND_CLASS, y=Wn[idx1], ntree=num_trees, seed=seed,
                           backend=be, edges=edges)
        rf2 = F.fit_forest(Xn[idx2], F.KIND_CLASS, y=Yn[idx2], ntree=num_trees, seed=seed + 1,
                           backend=be, edges=edges)
        ew = rf1.predict_proba(Xn)
        ey = rf2.predict_proba(Xn)
    return R.resid_on_resid(Yn - ey, Wn - ew)


def double_ml(Y, W, X, num_trees=100, seed=123, method="Double Machine Learning", device=None,
              comm=None):
    """E13 ``double_ml`` (ate_functions.R:372-389): positional halves, swapped, averaged
    tau and averaged SE (Q14)."""
    n = len(as_np(Y))
    h = n // 2
    idx1, idx2 = np.arange(h), np.arange(h, n)
    t1, s1 = chernozhukov(Y, W, X, idx1, idx2, num_trees, seed, device, comm)
    t2, s2 = chernozhukov(Y, W, X, idx2, idx1, num_trees, seed + 2, device, comm)
    return AteResult.make(method, (t1 + t2) / 2, (s1 + s2) / 2)


def causal_forest_ate(Y, W, X, num_trees=2000, seed=12345, method="Causal Forest(GRF)",
                      device=None, nuisance_trees=None, comm=None):
    """E15 (ate_replication.Rmd:250-272): grf causal forest; published row = AIPW
    ``estimate_average_effect``; diagnostics carry the "incorrect" mean-CATE ATE and
    sqrt(mean(var)) the reference prints (ate_replication.md:294)."""
    cf = F.causal_forest(as_np(X), as_np(Y), as_np(W), num_trees=num_trees, seed=seed,
                         nuisance_trees=nuisance_trees, backend=_backend(device), comm=comm)
    est, se = F.average_treatment_effect(cf)
    return AteResult.make(method, est, se, ate_bad=float(np.nanmean(cf.tau_oob)),
                          se_bad=float(np.sqrt(np.nanmean(cf.var_oob))))
