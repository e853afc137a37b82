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


def _rf_oob(Xn, y, num_trees, seed, dev, comm, splits="binned"):
    if comm is not None and comm.world_size > 1:
        fr = F.fit_forest_sharded(Xn, F.KIND_CLASS, num_trees, comm, y=y, seed=seed,
                                  backend=_backend(dev), splits=splits)
        return F.predict_tree_parallel(fr, comm, oob=True)
    return F.rf_classifier(Xn, y, num_trees=num_trees, seed=seed, backend=_backend(dev),
                           splits=splits).oob_proba()


def _device_bins(Xn, splits, dev):
    """(binned rows on the device, value table (vals, nval) device tensors or (None, None))
    -- graph-body inputs."""
    if splits == "exact":
        eb = F.exact_bins(Xn)
        de = eb.on(dev)
        return torch.from_numpy(eb.bin(Xn)).to(dev), de.vals, de.nval
    edges = F.bin_edges(Xn)
    return F.bin_matrix(Xn, *edges, dev), None, None


def _fit_class(Xb, ex, y, ntree, seed, tree_offset=0):
    """randomForest classifier on device bins: exact splits when a value table (vals, nval)
    is given."""
    if ex[0] is not None:
        return F.fit_forest_exact(Xb, F.DeviceExactBins(*ex), F.KIND_CLASS, y=y, ntree=ntree,
                                  seed=seed, tree_offset=tree_offset)
    return F.fit_forest_binned(Xb, (None, None), F.KIND_CLASS, y=y, ntree=ntree, seed=seed,
                               tree_offset=tree_offset)


def aipw_rf(Y, W, X, num_trees=100, bootstrap_se=False, B=1000, seed=1991, forest_seed=12325,
            compat="reference", method="Doubly Robust with Random Forest PS", device=None,
            dtype="f64", comm=None, graph=True, splits="auto"):
    """E8 ``doubly_robust`` (ate_functions.R:149-207): logistic outcome model (with the
    mutate_ quirk Q6 under compat="reference"), randomForest OOB propensity clipped (Q9).
    ``comm``: tree-parallel propensity forest over ranks (rows replicated, C05).
    ``splits``: "exact" = randomForest's split semantics (every distinct value, midpoint
    thresholds), "binned" = 256-bin histograms, "auto" = exact up to 65536 rows."""
    dev = resolve_device(device)
    Yn, Wn, Xn = as_np(Y), as_np(W), as_np(X)
    splits = F.resolve_splits(splits, len(Yn), Xn.shape[1])
    from ..parallel.comm import capturable
    if graph and capturable(comm) and dev.type == "cuda":
        # one hipGraph launch: outcome IRLS + counterfactual predictions, the propensity
        # forest (growth, OOB votes, clipping) and the AIPW score, over the binned matrix
        # (bin edges come from the data, so binning stays in front of the graph); with a
        # tree-parallel RCCL comm the OOB-vote all-reduce (C05) is captured in the graph
        from ..utils.graphs import estimator_graphs
        po = D._outcome_panel(Yn, Wn, Xn, dtype, dev)
        Xb, ev, en = _device_bins(Xn, splits, dev)
        y = torch.as_tensor(Yn, device=dev)
        w = torch.as_tensor(Wn, device=dev)
        cm = comm if comm is not None and comm.world_size > 1 else None
        out, g = estimator_graphs.run("aipw_rf", _aipw_rf_body, (po, Xb, y, w, ev, en),
                                      num_trees, forest_seed, compat, bootstrap_se, B, seed, cm)
        v = out.cpu().numpy()
        return AteResult.make(method, v[0], v[1], n_oob_nan=int(v[2]), hipgraph=g)
    mu0, mu1 = D.outcome_mu(Yn, Wn, Xn, counterfactual_quirk=(compat == "reference"),
                            device=dev, dtype=dtype)
    p_raw = _rf_oob(Xn, Wn, num_trees, forest_seed, dev, comm, splits)
    p = torch.as_tensor(p_raw, device=dev)
    from ..ops import stats as S
    S.clip_propensity_(p)
    return D.aipw_from_nuisances(method, Yn, Wn, p, mu0, mu1, bootstrap_se, B, seed, compat, dev,
                                 n_oob_nan=int(np.isnan(p_raw).sum()))


def _aipw_rf_body(po, Xb, y, w, ev, en, num_trees, forest_seed, compat, bootstrap_se, B, seed,
                  comm=None):
    """Device body of aipw_rf (no host sync): [ate, se, #OOB-NaN propensities]. ``comm``
    (world > 1): this rank grows its tree shard and the per-tree OOB vote sums are
    all-reduced (C05) before the vote shares are formed. ``ev, en``: device value table of
    the exact-split mode (None: 256-bin histograms)."""
    from ..ops import stats as S
    mu0, mu1 = D._outcome_fit(po, compat == "reference")
    ex = (ev, en)
    if comm is None:
        fr = _fit_class(Xb, ex, w, num_trees, forest_seed)
        p = fr.predict_state(Xb, True, fr.new_state(Xb.shape[1]), 7, host=False).clone()
    else:
        t0, cnt = F.tree_shard(num_trees, 1, comm.rank, comm.world_size)
        fr = _fit_class(Xb, ex, w, cnt, forest_seed, tree_offset=t0)
        n = Xb.shape[1]
        st = fr.new_state(n)
        fr.predict_state(Xb, True, st, 1, host=False)
        comm.all_reduce_(st[:2 * n])
        p = fr.predict_state(Xb, True, st, 4, host=False).clone()
    nan = torch.isnan(p).sum().double().reshape(1)
    S.clip_propensity_(p)
    res = D._aipw_core(y, w, p, mu0, mu1, bootstrap_se, B, seed, compat)
    return torch.cat([res, nan])


def _double_ml_body(Xb, y, w, ev, en, num_trees, seed):
    """Device body of double_ml (no host sync): both positional halves (Q14), [tau, se].
    ``ev, en``: device value table of the exact-split mode (bins of ALL rows, so the
    held-out half is classified by the midpoint rule), None: 256-bin histograms."""
    ex = (ev, en)
    n = Xb.shape[1]
    h = n // 2
    halves = []
    for (a0, a1), (b0, b1), sd in (((0, h), (h, n), seed), ((h, n), (0, h), seed + 2)):
        rf1 = _fit_class(Xb[:, a0:a1].contiguous(), ex, w[a0:a1], num_trees, sd)
        rf2 = _fit_class(Xb[:, b0:b1].contiguous(), ex, y[b0:b1], num_trees, sd + 1)
        ew = rf1.predict_state(Xb, False, rf1.new_state(n), 7, host=False)
        ey = rf2.predict_state(Xb, False, rf2.new_state(n), 7, host=False)
        yr, wr = y - ey, w - ew
        sww = wr @ wr                                  # lm(Y_resid ~ 0 + W_resid)
        tau = (wr @ yr) / sww
        rss = ((yr - tau * wr) ** 2).sum()
        halves.append(torch.stack([tau, torch.sqrt(rss / (n - 1) / sww)]))
    return (halves[0] + halves[1]) / 2


def _causal_forest_body(Xb, y, w, ev, en, num_trees, nt, seed, clip=None):
    """Device body of causal_forest_ate (models/forest.causal_forest + average_treatment_
    effect with grf defaults, no host sync): [AIPW ATE, SE, mean CATE, sqrt(mean var),
    min W.hat, max W.hat]. ``clip``: None = grf (no clipping), else W.hat clipped to
    [clip, 1 - clip] (compat="textbook").
    ``ev, en``: the exact mode's device value table (grf's exact split values), None:
    256-bin histograms. The orthogonalisation forests use ci.group.size = 1 (grf)."""
    p = Xb.shape[0]
    grf = dict(mtry=F.grf_mtry(p), min_node=5, sampling=1, honesty=True, mtry_poisson=True,
               alpha=0.05, sample_fraction=0.5)

    def oob(fr):
        return fr.predict_state(Xb, True, fr.new_state(Xb.shape[1]), 7, host=False)

    def grow(kind, ntree, sd, group, **kw):
        if ev is not None:
            return F.fit_forest_exact(Xb, F.DeviceExactBins(ev, en), kind, ntree=ntree, seed=sd,
                                      group=group, **grf, **kw)
        return F.fit_forest_binned(Xb, (None, None), kind, ntree=ntree, seed=sd, group=group,
                                   **grf, **kw)

    fy = grow(F.KIND_REG, nt, seed + 1, 1, r1=y)
    fw = grow(F.KIND_REG, nt, seed + 2, 1, r1=w)
    y_hat, w_hat = oob(fy), oob(fw)
    y_hat = torch.where(torch.isnan(y_hat), y.mean(), y_hat)
    w_hat = torch.where(torch.isnan(w_hat), w.mean(), w_hat)
    fc = grow(F.KIND_CAUSAL, num_trees, seed, 2, r1=w - w_hat, r2=y - y_hat)
    out = oob(fc)
    tau_oob, var_oob = out[:, 0], out[:, 1]
    w_res, y_res = w - w_hat, y - y_hat
    tau = torch.where(torch.isnan(tau_oob), torch.nanmean(tau_oob), tau_oob)
    what = w_hat if clip is None else w_hat.clamp(clip, 1 - clip)
    gamma = tau + w_res / (what * (1 - what)) * (y_res - tau * w_res)
    n = gamma.numel()
    return torch.stack([gamma.mean(), gamma.std(unbiased=True) / n ** 0.5,
                        torch.nanmean(tau_oob), torch.sqrt(torch.nanmean(var_oob)),
                        w_hat.min(), w_hat.max()])


def chernozhukov(Y, W, X, idx1, idx2, num_trees, seed=123, device=None, comm=None,
                 splits="auto"):
    """One half of ``double_ml`` (ate_functions.R:332-369): RF classifier for W on idx1,
    for Y on idx2, both predicted on all rows (in-sample for the training half, Q14).
    Bins (256-bin edges or the exact mode's value table) come from ALL rows."""
    be = _backend(device)
    Yn, Wn, Xn = as_np(Y), as_np(W), as_np(X)
    splits = F.resolve_splits(splits, len(Yn), Xn.shape[1])
    edges = F.exact_bins(Xn) if splits == "exact" else F.bin_edges(Xn)
    kw = dict(backend=be, edges=edges, splits=splits)
    if comm is not None and comm.world_size > 1:
        rf1 = F.fit_forest_sharded(Xn[idx1], F.KIND_CLASS, num_trees, comm, y=Wn[idx1], seed=seed,
                                   **kw)
        rf2 = F.fit_forest_sharded(Xn[idx2], F.KIND_CLASS, num_trees, comm, y=Yn[idx2],
                                   seed=seed + 1, **kw)
        ew = F.predict_tree_parallel(rf1, comm, X=Xn)
        ey = F.predict_tree_parallel(rf2, comm, X=Xn)
    else:
        rf1 = F.fit_forest(Xn[idx1], F.KIND_CLASS, y=Wn[idx1], ntree=num_trees, seed=seed, **kw)
        rf2 = F.fit_forest(Xn[idx2], F.KIND_CLASS, y=Yn[idx2], ntree=num_trees, seed=seed + 1,
                           **kw)
        ew = rf1.predict_proba(Xn)
        ey = rf2.predict_proba(Xn)
    return R.resid_on_resid(Yn - ey, Wn - ew)


def double_ml(Y, W, X, num_trees=100, seed=123, method="Double Machine Learning", device=None,
              comm=None, graph=True, splits="auto"):
    """E13 ``double_ml`` (ate_functions.R:372-389): positional halves, swapped, averaged
    tau and averaged SE (Q14). ``splits`` as in aipw_rf."""
    n = len(as_np(Y))
    h = n // 2
    dev = resolve_device(device)
    splits = F.resolve_splits(splits, n, as_np(X).shape[1])
    if graph and (comm is None or comm.world_size == 1) and dev.type == "cuda":
        # one hipGraph launch: the four forests, their predictions on all rows and both
        # residual-on-residual fits, over the binned matrix (edges from the data)
        from ..utils.graphs import estimator_graphs
        Xn = as_np(X)
        Xb, ev, en = _device_bins(Xn, splits, dev)
        y = torch.as_tensor(as_np(Y), device=dev)
        w = torch.as_tensor(as_np(W), device=dev)
        out, g = estimator_graphs.run("double_ml", _double_ml_body, (Xb, y, w, ev, en),
                                      num_trees, seed)
        v = out.cpu().numpy()
        return AteResult.make(method, v[0], v[1], hipgraph=g)
    idx1, idx2 = np.arange(h), np.arange(h, n)
    t1, s1 = chernozhukov(Y, W, X, idx1, idx2, num_trees, seed, device, comm, splits)
    t2, s2 = chernozhukov(Y, W, X, idx2, idx1, num_trees, seed + 2, device, comm, splits)
    return AteResult.make(method, (t1 + t2) / 2, (s1 + s2) / 2)


def causal_forest_ate(Y, W, X, num_trees=2000, seed=12345, method="Causal Forest(GRF)",
                      device=None, nuisance_trees=None, comm=None, graph=True, splits="auto",
                      compat="reference"):
    """E15 (ate_replication.Rmd:250-272): grf causal forest; published row = AIPW
    ``estimate_average_effect``; diagnostics carry the "incorrect" mean-CATE ATE and
    sqrt(mean(var)) the reference prints (ate_replication.md:294). ``splits``: "auto" =
    grf's exact split values up to 65,536 rows (df_mod), else 256-bin histograms.
    ``compat="reference"``: grf's AIPW without clipping W.hat (a poor-overlap warning, as
    grf); "textbook": W.hat clipped to [1e-6, 1 - 1e-6]."""
    dev = resolve_device(device)
    clip = None if compat == "reference" else F.AIPW_TEXTBOOK_CLIP
    splits = F.resolve_splits(splits, len(as_np(Y)), as_np(X).shape[1])
    if graph and (comm is None or comm.world_size == 1) and dev.type == "cuda":
        # one hipGraph launch: Y.hat / W.hat OOB regression forests, the honest causal
        # forest on the centred data, its OOB CATEs and the AIPW average effect
        from ..utils.graphs import estimator_graphs
        Xn = as_np(X)
        Xb, ev, en = _device_bins(Xn, splits, dev)
        y = torch.as_tensor(as_np(Y), device=dev)
        w = torch.as_tensor(as_np(W), device=dev)
        nt = nuisance_trees or max(50, num_trees // 4)
        out, g = estimator_graphs.run("causal_forest", _causal_forest_body, (Xb, y, w, ev, en),
                                      num_trees, nt, seed, clip)
        v = out.cpu().numpy()
        F.overlap_warning(float(v[4]), float(v[5]))
        return AteResult.make(method, v[0], v[1], ate_bad=float(v[2]), se_bad=float(v[3]),
                              hipgraph=g, splits=splits, w_hat_min=float(v[4]),
                              w_hat_max=float(v[5]))
    cf = F.causal_forest(as_np(X), as_np(Y), as_np(W), num_trees=num_trees, seed=seed,
                         nuisance_trees=nuisance_trees, backend=_backend(device), comm=comm,
                         splits=splits)
    est, se = F.average_treatment_effect(cf, clip)
    return AteResult.make(method, est, se, ate_bad=float(np.nanmean(cf.tau_oob)),
                          se_bad=float(np.sqrt(np.nanmean(cf.var_oob))),
                          w_hat_min=float(np.min(cf.w_hat)), w_hat_max=float(np.max(cf.w_hat)))
