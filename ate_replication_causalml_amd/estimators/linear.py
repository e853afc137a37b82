"""Device estimators built on Gram / IRLS / score kernels:
E1 naive, E2 OLS (Direct Method), E16 logistic propensity, E3 IPW, E4 PS-WLS,
E9 doubly-robust (logistic), E10 bootstrap SE.

Semantics follow ``ate_functions.R`` exactly (see reference/estimators.py for the
float64 CPU oracle and SURVEY.md §2.7); each function takes ``(Y, W, X)``.
Default precision is the fp64 parity panel (fp64 MFMA Gram), the right choice at
tutorial scale (N ~ 1e4, p = 21); ``dtype="f32"`` uses fp32 MFMA.

``dist=parallel.dist.DistContext(...)``: (Y, W, X) are this rank's row shard; group
moments, Gram matrices, IRLS statistics and score moments are all-reduced, and the
bootstrap replicates are sharded across ranks (all-gather of the estimates, C07).
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import stats as S
from ..ops.gram import gram
from ..ops.linalg import chol_solve, logistic_irls, predict
from ..ops.panel import build_panel
from ..utils.graphs import estimator_graphs
from ..result import AteResult
from .common import as_np, read_result, resolve_device


def _n(pan, dist):
    return dist.n_total if dist is not None else pan.n


def _graph_ok(graph, dist, t):
    return graph and dist is None and t.is_cuda


def naive(Y, W, method="naive", device=None, dist=None, graph=True):
    """E1 ``naive_ate`` (ate_functions.R:3-21)."""
    dev = resolve_device(device)
    y = torch.as_tensor(as_np(Y), device=dev)
    w = torch.as_tensor(as_np(W), device=dev)
    if _graph_ok(graph, dist, y):
        res, g = estimator_graphs.run("naive", lambda y_, w_: S.naive(y_, w_)[0], (y, w))
        return read_result(res, method, hipgraph=g)
    res, mom = S.naive(y, w)
    if dist is not None:
        res = S._naive_finalize(dist.sum_(mom.clone()).cpu())
    return read_result(res, method)


def _ols_body(pan, n=None):
    """Gram -> rank-revealing solve -> [ate, se, rank] (device-only, capturable)."""
    G = gram(pan)[0]
    return _ols_finish(pan, G, pan.n if n is None else n)


def _ols_finish(pan, G, n):
    cols = [pan.cols["one"], *pan.xcols, pan.cols["W"]]
    r = chol_solve(G, cols, pan.cols["Y"])
    return torch.stack([r.beta[-1], torch.sqrt(r.aux[1] / (n - r.aux[0]) * r.invdiag[-1]),
                        r.aux[0]])


def ols(Y, W, X, method="Direct Method", device=None, dtype="f64", dist=None, graph=True):
    """E2 ``ate_condmean_ols`` (ate_functions.R:25-39): lm(Y ~ covariates + W)."""
    dev = resolve_device(device)
    pan = build_panel(as_np(X), as_np(W), as_np(Y), dtype=dtype, device=dev)
    diag = {}
    if _graph_ok(graph, dist, pan.data):
        out, diag["hipgraph"] = estimator_graphs.run("ols", _ols_body, (pan,))
    else:
        G = gram(pan)[0]
        if dist is not None:
            dist.sum_(G)
        out = _ols_finish(pan, G, _n(pan, dist))
    v = out.cpu().numpy()
    return AteResult.make(method, v[0], v[1], rank=int(v[2]), **diag)


def propensity_logistic(W, X, device=None, dtype="f64", return_panel_order=False, dist=None):
    """E16: glm(W ~ covariates, binomial) fitted values (ate_replication.Rmd:165-168)."""
    dev = resolve_device(device)
    pan = _propensity_panel(W, X, dtype, dev)
    fit = _propensity_fit(pan, dist)
    if return_panel_order:
        return fit.mu, pan
    return pan.scatter_rows(fit.mu)


def _propensity_panel(W, X, dtype, dev):
    return build_panel(as_np(X), as_np(W), None, dtype=dtype, device=dev, extra_cols=("z",))


def _propensity_fit(pan, dist=None):
    cols = [pan.cols["one"], *pan.xcols]
    return logistic_irls(pan, cols, pan.cols["W"], pan.cols["z"], dist=dist)


def propensity_lasso(W, X, seed=1991, nfolds=10, fold_stream=7, device=None, dtype="f64"):
    """E7 ``prop_score_lasso`` (ate_functions.R:133-146): binomial cv.glmnet, predicted
    response at lambda.1se (Q5); folds = Philox fold ids (stream 7) as the reference."""
    from ..ops.lognet import cv_lognet
    from ..parallel import rng
    dev = resolve_device(device)
    Wn = as_np(W)
    fid = rng.fold_ids(len(Wn), nfolds, seed, fold_stream)
    pan = build_panel(as_np(X), None, Wn, folds=fid, dtype=dtype, device=dev)
    cv = cv_lognet(pan, pan.xcols, pan.cols["Y"]).check()
    cols = [pan.cols["one"], *pan.xcols]
    mu = predict(pan, cols, cv.coef_1se.to(dev, torch.float64).contiguous(), link="logit")
    return pan.scatter_rows(mu)


def ipw(Y, W, X, p, method="Propensity_Weighting", compat="reference", device=None, dtype="f64",
        dist=None, graph=True):
    """E3 ``prop_score_weight`` (ate_functions.R:44-63) with the full-frame projection
    design under compat="reference" (Q25; see reference.estimators.ipw_design)."""
    dev = resolve_device(device)
    Yn, Wn, Xn = as_np(Y), as_np(W), as_np(X)
    pt = torch.as_tensor(as_np(p), device=dev)
    y = torch.as_tensor(Yn, device=dev)
    w = torch.as_tensor(Wn, device=dev)
    x = torch.as_tensor(Xn, device=dev)
    ps = w - pt
    tau = ps * y / (pt * (1 - pt))
    frame = torch.cat([x, y[:, None], w[:, None], pt[:, None], tau[:, None], ps[:, None]], 1) \
        if compat == "reference" else x
    d = frame * ps[:, None]
    pan = build_panel(d.cpu().numpy(), None, tau.cpu().numpy(), dtype=dtype, device=dev)
    if _graph_ok(graph, dist, pan.data):
        res, g = estimator_graphs.run("ipw", _ipw_body, (pan,))
        return read_result(res, method, hipgraph=g)
    G = gram(pan)[0]
    if dist is not None:
        dist.sum_(G)
    return read_result(_ipw_finish(pan, G, _n(pan, dist)), method)


def _ipw_body(pan):
    return _ipw_finish(pan, gram(pan)[0], pan.n)


def _ipw_finish(pan, G, n):
    cols = [pan.cols["one"], *pan.xcols]
    r = chol_solve(G, cols, pan.cols["Y"])
    ate = G[pan.cols["one"], pan.cols["Y"]] / n
    se = torch.sqrt(r.aux[1] / n) / np.sqrt(n)
    return torch.stack([ate, se])


def ipw_wls(Y, W, p, method="Propensity_Regression", device=None, dtype="f64", dist=None,
            graph=True):
    """E4 ``prop_score_ols`` (ate_functions.R:67-86): WLS of Y on W, weights W/p+(1-W)/(1-p)."""
    dev = resolve_device(device)
    Wn, pn = as_np(W), as_np(p)
    wts = Wn / pn + (1 - Wn) / (1 - pn)
    pan = build_panel(Wn[:, None], None, as_np(Y), dtype=dtype, device=dev)
    wt = pan.gather_rows(torch.as_tensor(wts, device=dev).to(pan.dtype))
    if _graph_ok(graph, dist, pan.data):
        res, g = estimator_graphs.run("ipw_wls", _wls_body, (pan, wt))
        return read_result(res, method, hipgraph=g)
    G = gram(pan, wt)[0]
    if dist is not None:
        dist.sum_(G)
    return read_result(_wls_finish(pan, G, _n(pan, dist)), method)


def _wls_body(pan, wt):
    return _wls_finish(pan, gram(pan, wt)[0], pan.n)


def _wls_finish(pan, G, n):
    cols = [pan.cols["one"], pan.xcols[0]]
    r = chol_solve(G, cols, pan.cols["Y"])
    se = torch.sqrt(r.aux[1] / (n - r.aux[0]) * r.invdiag[1])
    return torch.stack([r.beta[1], se])


def _outcome_panel(Y, W, X, dtype, dev):
    return build_panel(np.column_stack([as_np(X), as_np(W)]), None, as_np(Y), dtype=dtype,
                       device=dev, extra_cols=("z",))


def _outcome_fit(pan, counterfactual_quirk, dist=None):
    """Outcome logistic GLM on its panel -> (mu0, mu1) in original row order."""
    cols = [pan.cols["one"], *pan.xcols]
    fit = logistic_irls(pan, cols, pan.cols["Y"], pan.cols["z"], dist=dist)
    if counterfactual_quirk:
        mu = pan.scatter_rows(fit.mu)
        return mu, mu.clone()
    widx = len(cols) - 1
    mu1 = predict(pan, cols, fit.beta, override_idx=widx, override_val=1.0, link="logit")
    mu1 = pan.scatter_rows(mu1.clone())
    mu0 = predict(pan, cols, fit.beta, override_idx=widx, override_val=0.0, link="logit")
    mu0 = pan.scatter_rows(mu0.clone())
    return mu0, mu1


def outcome_mu(Y, W, X, counterfactual_quirk, device=None, dtype="f64", dist=None):
    """Outcome GLM Y ~ covariates + W (Q24); mu1/mu0 with W overridden to 1/0, or both
    equal to mu(x, W_obs) under the ``mutate_("W = 1")`` quirk (Q6)."""
    pan = _outcome_panel(Y, W, X, dtype, resolve_device(device))
    return _outcome_fit(pan, counterfactual_quirk, dist)


def aipw_from_nuisances(method, Y, W, p, mu0, mu1, bootstrap_se=False, B=1000, seed=1991,
                        compat="reference", device=None, dist=None, **diag):
    dev = resolve_device(device)
    y = torch.as_tensor(as_np(Y), device=dev)
    w = torch.as_tensor(as_np(W), device=dev)
    p = p.to(dev).double()
    if dist is None:
        return read_result(_aipw_core(y, w, p, mu0.to(dev), mu1.to(dev), bootstrap_se, B, seed,
                                      compat), method, **diag)
    res, mom = S.aipw(w, y, p, mu0.to(dev), mu1.to(dev), compat=compat)
    res = S._aipw_finalize(dist.sum_(mom.clone()))
    if bootstrap_se:
        e1, e2 = S.aipw_terms(w, y, p, mu0.to(dev), mu1.to(dev), compat)
        taus = bootstrap_sharded(e1, e2, B, seed, dist)
        res = torch.stack([res[0], taus.std(unbiased=True).to(res.device)])
    return read_result(res, method, **diag)


def _aipw_glm_body(po, pp, y, w, bootstrap_se, B, seed, compat, dist=None):
    """Both IRLS fits (their per-iteration Gram / deviance all-reduces over row shards
    included, C01/C02), counterfactual predictions and the AIPW score (moments all-reduced,
    C06; bootstrap replicates sharded, C07): device-only, capturable."""
    mu0, mu1 = _outcome_fit(po, False, dist)
    p = pp.scatter_rows(_propensity_fit(pp, dist).mu)
    if dist is None or dist.world == 1:
        return _aipw_core(y, w, p, mu0, mu1, bootstrap_se, B, seed, compat)
    res, mom = S.aipw(w, y, p, mu0, mu1, compat=compat)
    res = S._aipw_finalize(dist.sum_(mom.clone()))
    if bootstrap_se:
        e1, e2 = S.aipw_terms(w, y, p, mu0, mu1, compat)
        taus = bootstrap_sharded(e1, e2, B, seed, dist)
        res = torch.stack([res[0], taus.std(unbiased=True).to(res.device)])
    return res


def _aipw_core(y, w, p, mu0, mu1, bootstrap_se, B, seed, compat):
    """AIPW [ate, se] from nuisances on one device (capturable: native score / bootstrap
    kernels, no host sync)."""
    res, _ = S.aipw(w, y, p, mu0, mu1, compat=compat)
    if bootstrap_se:
        e1, e2 = S.aipw_terms(w, y, p, mu0, mu1, compat)
        taus = S.bootstrap_multinomial(e1.contiguous(), e2.contiguous(), B, seed)
        res = torch.stack([res[0], taus.std(unbiased=True).to(res.device)])
    return res


def bootstrap_sharded(e1, e2, B, seed, dist):
    """E10 with the B replicates split across ranks (C07) for ROW-SHARDED scores: the
    terms are all-gathered (N doubles x2) and handed to ``bootstrap_replicates``."""
    e1f = dist.gather_rows(e1.double().contiguous())
    e2f = dist.gather_rows(e2.double().contiguous())
    return bootstrap_replicates(e1f, e2f, B, seed, dist.comm)


def bootstrap_replicates(e1, e2, B, seed, comm=None, b_start=0):
    """tau_b for b_start <= b < b_start + B with the replicates sharded over ``comm``
    (rows replicated on every rank): rank r evaluates its slice with the same
    global-index Philox draws as one device, then the estimates are all-gathered in rank
    order (C07). ``b_start`` lets a long run resample in checkpointed ranges."""
    from ..parallel.dist import shard_range
    world = comm.world_size if comm is not None else 1
    rank = comm.rank if comm is not None else 0
    b0, nb = shard_range(B, rank, world)
    b0 += b_start
    mine = S.bootstrap_multinomial(e1.contiguous(), e2.contiguous(), nb, seed, b0=b0) \
        if nb else torch.empty(0, dtype=torch.float64, device=e1.device)
    if world == 1:
        return mine
    mb = shard_range(B, 0, world)[1]
    buf = torch.zeros(mb, dtype=torch.float64, device=e1.device)
    buf[:nb] = mine.to(buf.device)
    parts = comm.all_gather(buf)
    return torch.cat([pp[:shard_range(B, r, world)[1]] for r, pp in enumerate(parts)])


def aipw_glm(Y, W, X, bootstrap_se=False, B=1000, seed=1991, compat="reference",
             method="Doubly Robust with logistic regression PS", device=None, dtype="f64",
             dist=None, graph=True):
    """E9 ``doubly_robust_glm`` (ate_functions.R:211-264). On a GPU both IRLS fits, the
    counterfactual predictions, the AIPW score moments and the optional bootstrap run as
    ONE captured hipGraph (replayed for later calls of the same shape); with ``dist``
    over RCCL the all-reduces are inside that graph."""
    dev = resolve_device(device)
    if graph and (dist is None or dist.capturable) and dev.type == "cuda":
        po = _outcome_panel(Y, W, X, dtype, dev)
        pp = _propensity_panel(W, X, dtype, dev)
        y = torch.as_tensor(as_np(Y), device=dev)
        w = torch.as_tensor(as_np(W), device=dev)

        res, g = estimator_graphs.run("aipw_glm", _aipw_glm_body, (po, pp, y, w), bootstrap_se,
                                      B, seed, compat, dist)
        return read_result(res, method, hipgraph=g)
    mu0, mu1 = outcome_mu(Y, W, X, counterfactual_quirk=False, device=device, dtype=dtype,
                          dist=dist)
    p = propensity_logistic(W, X, device=device, dtype=dtype, dist=dist)
    return aipw_from_nuisances(method, Y, W, p, mu0, mu1, bootstrap_se, B, seed, compat, device,
                               dist=dist)
