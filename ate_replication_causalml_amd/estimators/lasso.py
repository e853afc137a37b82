"""Device LASSO-family estimators: E5 single-equation LASSO, E6 usual LASSO,
E11 Belloni post-double-selection, and the K-fold cross-fit DML (partially
linear model) with CV-LASSO nuisances — the north-star estimator.

All LASSO fits run on the per-fold Gram stack (K01, one pass over the panel)
followed by on-device coordinate descent, CV loss and lambda selection (K08/K09).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _native
from ..ops import stats as S
from ..ops.devconst import const
from ..ops.enet import cv_enet_gaussian
from ..ops.gram import gram
from ..ops.linalg import chol_solve, chol_solve_active
from ..ops.panel import build_panel, dtype_code
from ..parallel import rng
from ..reference.estimators import lambda_interp
from ..result import AteResult
from ..utils.graphs import estimator_graphs
from .common import as_np, read_result, resolve_device


def _fold_ids(n, K, seed, stream, dist):
    return dist.fold_ids(K, seed, stream) if dist is not None else rng.fold_ids(n, K, seed, stream)


def _sharded_gram(pan, dist):
    """Per-segment Gram stack, all-reduced over row shards; + global segment counts."""
    G = gram(pan)
    if dist is None:
        return G, None
    dist.sum_(G)
    return G, global_seg_counts(pan, dist.comm)


def _lasso_w_panel(Y, W, X, seed, nfolds, fold_stream, device, dtype, dist=None):
    dev = resolve_device(device)
    Xn = np.column_stack([as_np(X), as_np(W)])
    fid = _fold_ids(Xn.shape[0], nfolds, seed, fold_stream, dist)
    return build_panel(Xn, None, as_np(Y), folds=fid, dtype=dtype, device=dev)


def _lasso_w_cv(pan, pf_w, G, counts=None):
    pf = np.r_[np.ones(len(pan.xcols) - 1), pf_w]
    return cv_enet_gaussian(G, pan, pan.xcols, [pan.cols["Y"]], penalty_factor=pf,
                            seg_counts=counts)


def _lasso_w_body(pan, pf_w, dist=None, counts=None):
    """Gram stack (all-reduced over row shards with ``dist``: C01) -> CV-LASSO path ->
    [coef of W at lambda.1se, lambda.1se, min fold passes] (device-only: the fold
    truncation flag travels with the result; ``counts`` = global rows per segment)."""
    G = gram(pan)
    if dist is not None:
        dist.sum_(G)
    cv = _lasso_w_cv(pan, pf_w, G, None if counts is None else np.asarray(counts))
    lam = cv.lambdas[0].gather(0, cv.sel[0, 1:2].long())
    fnp = cv.fold_npass.min().double().reshape(1) if cv.fold_npass is not None else \
        torch.zeros(1, dtype=torch.float64, device=lam.device)
    return torch.cat([cv.coef_1se[0, -1:].double(), lam.double(), fnp])


def _lasso_w(Y, W, X, pf_w, seed, nfolds, fold_stream, method, device, dtype, dist, graph):
    pan = _lasso_w_panel(Y, W, X, seed, nfolds, fold_stream, device, dtype, dist)
    if graph and (dist is None or dist.capturable) and pan.data.is_cuda:
        # row shards over RCCL: the Gram all-reduce is captured inside the graph
        counts = None if dist is None else tuple(global_seg_counts(pan, dist.comm).tolist())
        out, g = estimator_graphs.run("lasso_w", _lasso_w_body, (pan,), float(pf_w), dist,
                                      counts)
        v = out.cpu().numpy()
        if v[2] < 0:
            from ..utils.guards import NumericalError
            raise NumericalError("CV fold path timed out waiting for its full-data lambda "
                                 "sequence; selection is invalid")
        return AteResult.make(method, float(v[0]), None, lambda_1se=float(v[1]), hipgraph=g)
    G, counts = _sharded_gram(pan, dist)
    cv = _lasso_w_cv(pan, pf_w, G, counts).check()
    return AteResult.make(method, float(cv.coef_1se[0, -1]), None,
                          lambda_1se=float(cv.lambdas[0, int(cv.sel[0, 1])]))


def lasso_single(Y, W, X, seed=1991, nfolds=10, fold_stream=5, method="Single-equation LASSO",
                 device=None, dtype="f64", dist=None, graph=True):
    """E5 ``ate_condmean_lasso`` (ate_functions.R:89-108): W unpenalised, coef at lambda.1se.
    On a GPU: one hipGraph launch per call after the first (utils/graphs.GraphCache)."""
    return _lasso_w(Y, W, X, 0.0, seed, nfolds, fold_stream, method, device, dtype, dist, graph)


def lasso_usual(Y, W, X, seed=1991, nfolds=10, fold_stream=6, method="Usual LASSO", device=None,
                dtype="f64", dist=None, graph=True):
    """E6 ``ate_lasso`` (ate_functions.R:111-130): W penalised."""
    return _lasso_w(Y, W, X, 1.0, seed, nfolds, fold_stream, method, device, dtype, dist, graph)


def interaction_expand(x: torch.Tensor) -> torch.Tensor:
    """K21 (small p): [x, x_c1 * x_c2 for all ordered pairs incl. squares] (Q10);
    a HIP kernel on device tensors (ops/prep.py)."""
    from ..ops.prep import interactions
    return interactions(x)


def _interp_at(lams: torch.Tensor, nlam: torch.Tensor, path: torch.Tensor, s: torch.Tensor):
    """Device twin of reference.estimators.lambda_interp + coef_at: the coefficient path
    [L, p+1] linearly interpolated in lambda at ``s`` over the first ``nlam`` lambdas (no
    host sync, fixed shapes: capturable)."""
    L = lams.numel()
    k = nlam.long().clamp(min=1)
    ar = torch.arange(L, device=lams.device)
    valid = ar < k
    lam0 = lams[0]
    lamk = lams.gather(0, (k - 1).reshape(1))[0]
    den = lam0 - lamk
    single = den == 0
    dsafe = torch.where(single, torch.ones_like(den), den)
    sfrac = ((lam0 - s) / dsafe).clamp(0.0, 1.0)
    ln = torch.where(valid, (lam0 - lams) / dsafe, torch.full_like(lams, 2.0))
    left = ((ln <= sfrac) & valid).sum().clamp(min=1) - 1
    ln_l = ln.gather(0, left.reshape(1))[0]
    exact = (ln_l == sfrac) | single | (left + 1 >= k)
    right = torch.where(exact, left, left + 1)
    ln_r = ln.gather(0, right.reshape(1))[0]
    gap = ln_l - ln_r
    frac = torch.where(exact | (gap.abs() < np.finfo(float).eps), torch.ones_like(sfrac),
                       (sfrac - ln_r) / torch.where(gap == 0, torch.ones_like(gap), gap))
    # index_select, not path[left]: a 0-dim tensor index would be read on the host
    return (path.index_select(0, left.reshape(1))[0] * frac
            + path.index_select(0, right.reshape(1))[0] * (1 - frac))


def _belloni_body(panw, pany, panpost, compat):
    """E11 as one device function (GraphCache): the two CV-LASSO fits on the interaction
    panels, the Q11-Q13 selection as a column mask (W's lambda.min for both paths, positive
    coefficients, the one-column index shift), and the post-selection OLS on [one, the
    selected columns in natural order, W]: a fixed-length device column list with a device
    active count (ops/linalg.chol_solve_active). W's coefficient and SE do not depend on
    the design's column order, so this equals the host path's union-ordered design up to
    rounding.
    Returns [ate, se, n_selected, rank, min fold passes]."""
    cws = cv_enet_gaussian(gram(panw), panw, panw.xcols, [panw.cols["Y"]])
    cys = cv_enet_gaussian(gram(pany), pany, pany.xcols, [pany.cols["Y"]])
    q = len(panw.xcols)
    s = cws.lambdas[0].gather(0, cws.sel[0, 0:1].long())[0]
    bw = _interp_at(cws.lambdas[0], cws.nlam[0], cws.coef_path[0].double(), s)[1:]
    if compat == "reference":
        by = _interp_at(cys.lambdas[0], cys.nlam[0], cys.coef_path[0].double(), s)[1:]
        pos = (bw > 0) | (by > 0)
        keep = torch.cat([pos[1:], torch.zeros(1, dtype=torch.bool, device=pos.device)])
    else:
        sy = cys.lambdas[0].gather(0, cys.sel[0, 0:1].long())[0]
        by = _interp_at(cys.lambdas[0], cys.nlam[0], cys.coef_path[0].double(), sy)[1:]
        keep = (bw != 0) | (by != 0)
    G = gram(panpost)[0]
    dev = G.device
    # design = [one, selected x (natural order), W | unselected x]: a fixed-length column
    # list with the active count on the device (ops/linalg.chol_solve_active)
    xc = const(panpost.xcols[:q], torch.int32, dev)
    ki = keep.long()
    nsel = ki.sum()
    pos = torch.where(keep, ki.cumsum(0), 1 + nsel + (1 - ki).cumsum(0))
    wpos = (1 + nsel).reshape(1)
    dest = torch.cat([const([0], torch.int64, dev), pos, wpos])
    src = torch.cat([const([panpost.cols["one"]], torch.int32, dev), xc,
                     const([panpost.xcols[q]], torch.int32, dev)])
    cols = torch.empty(q + 2, dtype=torch.int32, device=dev).index_copy(0, dest, src)
    kact = (2 + nsel).to(torch.int32)
    r = chol_solve_active(G, cols, kact, panpost.cols["Y"])
    b_w = r.beta.gather(0, wpos)[0]
    se = torch.sqrt(r.aux[1] / (panpost.n - r.aux[0]) * r.invdiag.gather(0, wpos)[0])
    fnp = torch.stack([cws.fold_npass.min(), cys.fold_npass.min()]).min().double() \
        if cws.fold_npass is not None else torch.zeros((), dtype=torch.float64, device=dev)
    return torch.stack([b_w.double(), se.double(), nsel.double(), r.aux[0].double(), fnp])


def belloni(Y, W, X, seed=1991, nfolds=10, compat="reference", method="Belloni et.al",
            device=None, dtype="f64", dist=None, graph=True):
    """E11 ``belloni`` (ate_functions.R:286-328) with quirks Q10-Q13.

    On a GPU without row sharding: one hipGraph launch per call after the first
    (utils/graphs.GraphCache over _belloni_body); otherwise the selection is read on
    the host and the post-selection design is the union-ordered column list."""
    dev = resolve_device(device)
    Yn, Wn = as_np(Y), as_np(W)
    xint = interaction_expand(torch.as_tensor(as_np(X), device=dev))   # stays on the device
    n, q = xint.shape
    if graph and dist is None and dev.type == "cuda":
        panw = build_panel(xint, None, Wn, folds=_fold_ids(n, nfolds, seed, 8, None), dtype=dtype,
                           device=dev)
        pany = build_panel(xint, None, Yn, folds=_fold_ids(n, nfolds, seed, 9, None), dtype=dtype,
                           device=dev)
        post = torch.cat([xint, torch.as_tensor(Wn, dtype=torch.float64, device=dev)[:, None]], 1)
        panpost = build_panel(post, None, Yn, dtype=dtype, device=dev)
        out, g = estimator_graphs.run("belloni", _belloni_body, (panw, pany, panpost), compat)
        v = out.cpu().numpy()
        if v[4] < 0:
            from ..utils.guards import NumericalError
            raise NumericalError("CV fold path timed out waiting for its full-data lambda "
                                 "sequence; selection is invalid")
        return AteResult.make(method, float(v[0]), float(v[1]), n_selected=int(round(v[2])),
                              rank=int(round(v[3])), hipgraph=g)
    fits = []
    for target, stream in ((Wn, 8), (Yn, 9)):
        fid = _fold_ids(n, nfolds, seed, stream, dist)
        pan = build_panel(xint, None, target, folds=fid, dtype=dtype, device=dev)
        G, counts = _sharded_gram(pan, dist)
        fits.append((pan, G, cv_enet_gaussian(G, pan, pan.xcols, [pan.cols["Y"]],
                                              seg_counts=counts).check()))
    (_, _, cw), (_, _, cy) = fits
    s = float(cw.lambdas[0, int(cw.sel[0, 0])])
    lw = cw.lambdas[0, :int(cw.nlam[0])].cpu().numpy()
    ly = cy.lambdas[0, :int(cy.nlam[0])].cpu().numpy()
    pw = cw.coef_path[0, :len(lw)].cpu().numpy()
    py = cy.coef_path[0, :len(ly)].cpu().numpy()

    def coef_at(lams, path, s_):
        l, r, f = lambda_interp(lams, s_)
        return path[l] * f + path[r] * (1 - f)

    bw = coef_at(lw, pw, s)[1:]
    by = coef_at(ly, py, s if compat == "reference" else float(cy.lambdas[0, int(cy.sel[0, 0])]))[1:]
    if compat == "reference":
        union = []
        for v in np.concatenate([np.flatnonzero(bw > 0) + 1, np.flatnonzero(by > 0) + 1]):
            if int(v) not in union:
                union.append(int(v))
        cols = [v - 2 for v in union if v - 1 >= 1]        # Q13 shift, index 0 dropped
    else:
        cols = sorted(set(np.flatnonzero(bw != 0)) | set(np.flatnonzero(by != 0)))
    # post-selection OLS: y ~ 1 + x_int[:, cols] + W
    sel_x = torch.cat([xint[:, torch.as_tensor(cols, dtype=torch.long, device=xint.device)],
                       torch.as_tensor(Wn, dtype=torch.float64, device=xint.device)[:, None]], 1)
    pan = build_panel(sel_x, None, Yn, dtype=dtype, device=dev)
    G = gram(pan)[0]
    if dist is not None:
        dist.sum_(G)
    dcols = [pan.cols["one"], *pan.xcols]
    r = chol_solve(G, dcols, pan.cols["Y"])
    n_all = dist.n_total if dist is not None else pan.n
    se = torch.sqrt(r.aux[1] / (n_all - r.aux[0]) * r.invdiag[-1])
    return read_result(torch.stack([r.beta[-1], se]), method, n_selected=len(cols),
                       rank=int(r.aux[0]))


# ---------------------------------------------------------------- K-fold DML (PLR)
def global_seg_counts(pan, comm):
    """Rows per segment summed over ranks (host ints; one tiny all-reduce)."""
    c = torch.as_tensor(np.asarray(pan.seg_nreal, dtype=np.float64))
    if comm is not None and comm.world_size > 1:
        dev = pan.device
        t = c.to(dev)
        comm.all_reduce_(t)
        c = t.cpu()
    return c.numpy()


EXACT_BLOCK = 16384  # rows per Gram chunk in exact mode (synthetic_panel(align=EXACT_BLOCK))


def dml_residual_terms(pan, coef: torch.Tensor, rows: int = 1 << 20) -> torch.Tensor:
    """Per-row orthogonal-score terms [ld, 7] of the held-out residuals (the summands of
    dml_moments; padding rows all zero), computed with torch in row blocks (exact mode:
    the terms, not their order-dependent sums, are reduced)."""
    K = coef.shape[0]
    Xc = pan.colmajor()
    dev = Xc.device
    bf = pan.dtype == torch.bfloat16
    xc = torch.as_tensor(pan.xcols, dtype=torch.long, device=dev)
    out = []
    for k in range(K):
        r0, r1 = (int(v) for v in pan.seg_bounds[k])
        for a in range(r0, r1, rows):
            b = min(r1, a + rows)
            blk = Xc[:, a:b]
            valid = (blk[pan.cols["one"]] != 0).double()    # padding rows: all terms 0
            xs = blk.index_select(0, xc).double()
            y = blk[pan.cols["Y_hi"]].double() + blk[pan.cols["Y_lo"]].double() if bf else \
                blk[pan.cols["Y"]].double()
            w = blk[pan.cols["W_hi"]].double() + blk[pan.cols["W_lo"]].double() if bf else \
                blk[pan.cols["W"]].double()
            yr = y - (coef[k, 0, 0] + coef[k, 0, 1:].double() @ xs)
            wr = w - (coef[k, 1, 0] + coef[k, 1, 1:].double() @ xs)
            yr, wr = yr * valid, wr * valid         # (no boolean indexing: capturable)
            w2 = wr * wr
            out.append(torch.stack([wr * yr, w2, yr * yr * w2, yr * w2 * wr, w2 * w2,
                                    valid, yr * yr], 1))
    return torch.cat(out)


_TRI: dict = {}


def _tri_index(P: int, device):
    """Flat indices of the upper triangle (i <= j) of a P x P matrix and of the mirrored
    entries (j, i), row-major, cached per (P, device)."""
    key = (P, str(device))
    t = _TRI.get(key)
    if t is None:
        i, j = np.triu_indices(P)
        t = (torch.as_tensor(i * P + j, dtype=torch.int64).to(device),
             torch.as_tensor(j * P + i, dtype=torch.int64).to(device))
        _TRI[key] = t
    return t


def allreduce_sym_(comm, t: torch.Tensor) -> torch.Tensor:
    """In-place sum over ranks of a stack of symmetric P x P matrices (``t``: [..., P, P],
    contiguous), moving only the upper triangles (half the ring bytes of a full
    all-reduce); the lower triangle is mirrored from the reduced upper one, so the result
    is exactly symmetric."""
    P = t.shape[-1]
    up, lo = _tri_index(P, t.device)
    v = t.view(-1, P * P)
    buf = v.index_select(1, up)
    comm.all_reduce_(buf)
    v.index_copy_(1, up, buf)
    v.index_copy_(1, lo, buf)
    return t


def dml_phases(pan, folds: int, lambda_rule="min", comm=None, seg_counts=None, G=None,
               shard_paths=True, exact=False):
    """The cross-fit DML-PLR step as phases for utils.graphs.SegmentedStep:

    A  per-fold Gram stack (K01): tile kernel, then slab reduce     device (two phases)
    C01 all-reduce of the Gram stack over row shards               collective (world > 1)
    B  CV-LASSO paths for 5 folds x {Y, W} + inner CV, lambda.min
       selection (K08/K09)                                         device
    C08 all-reduce of the per-fold coefficients (world > 1, sharded paths)  collective
    B' fused held-out residual moments                             device
    C06 all-reduce of the 7 score moments                          collective (world > 1)
    C  theta / SE (fp64, on device)                                device

    The collectives are RCCL all-reduces on the current stream: utils.graphs.SegmentedStep
    captures them inside the step's graph (gloo ones run eagerly between graph segments).

    shard_paths (world > 1): the path solves are the N-independent part of the step, so
    instead of every rank repeating all of them, rank r solves the outer folds
    k = r, r + world, ... (each outer fold's full-data and inner-CV problems together)
    and the coefficients are summed over ranks (zeros elsewhere, so the sum is exact and
    the result equals the unsharded step bit for bit). Each rank's path launch then
    holds a fifth (or less) of the CUs it would, and the Gram beside it runs faster.

    Every phase maps a state dict to a state dict; device phases touch only tensors
    whose storage is static across calls, so the whole step can be captured.

    exact (block-aligned panels, synthetic_panel(align=EXACT_BLOCK)): the fold Gram stack
    is reduced as int64 limbs of per-block partials and all-reduced as integers, and the
    score moments are exact sums of per-row terms (ops/exact.py): ATE and SE are the SAME
    BITS at every world size, at the cost of a residual pass in torch."""
    from ..utils.graphs import Collective
    dist = comm is not None and comm.world_size > 1
    if dist and seg_counts is None:
        seg_counts = global_seg_counts(pan, comm)
    K = folds
    full_sets = [[s for s in range(K) if s != k] for k in range(K)]
    ycols = [pan.cols["Y"], pan.cols["W"]]
    sharded = dist and shard_paths
    mine = [k for k in range(K) if k % comm.world_size == comm.rank] if sharded else list(range(K))
    p1 = len(pan.xcols) + 1

    n_rows = int(np.asarray(seg_counts if seg_counts is not None else pan.seg_nreal).sum())
    if exact:
        # limb range guard, once per layout and agreed over ranks (a rank raising alone
        # would leave its peers blocked in the limb all-reduce): here, eagerly on every
        # rank, not inside the (captured) Gram phase
        from ..ops.gram import check_exact_range
        check_exact_range(pan, n_rows, comm=comm if dist else None)

    def phase_gram(_):
        if exact:
            return {"GX": gram(pan, stage="tiles", exact=True, n_total=n_rows, checked=True)}
        return {"G": gram(pan, stage="tiles") if G is None else G}

    def phase_gram_reduce(st):
        if exact:
            return {"GX": gram(pan, stage="reduce", exact=True)}
        return st if G is not None else {"G": gram(pan, stage="reduce", out=st["G"])}

    def phase_from_limbs(st):
        from ..ops.exact import from_limbs
        return {**st, "G": from_limbs(st["GX"])}

    native_exact = pan.data.is_cuda and pan.dtype == torch.bfloat16

    def phase_terms(st):
        from ..ops.exact import column_amax
        if native_exact:       # csrc/dml.hip exact mode 1: per-block max |term|, no row buffer
            part = _exact_resid(pan, st["coef"], 1, None)
            return {**st, "amax": part.view(-1, 7).amax(0)}
        terms = dml_residual_terms(pan, st["coef"])
        return {**st, "terms": terms, "amax": column_amax(terms)}

    def phase_limbs(st):
        from ..ops.exact import _scale_exp, sum_limbs
        if native_exact:       # mode 2: per-block int64 limb sums at the global scale
            sh = _scale_exp(st["amax"], n_rows).contiguous()
            part = _exact_resid(pan, st["coef"], 2, sh).view(torch.int64).view(-1, 14).sum(0)
            return {**st, "limbs": torch.stack([part[:7], part[7:]])}
        return {**st, "limbs": sum_limbs(st["terms"], st["amax"], n_rows)}

    def phase_mom_exact(st):
        from ..ops.exact import finish_limbs
        return {**st, "mom": finish_limbs(st["limbs"], st["amax"], n_rows)}

    def fit(st):
        if not mine:
            return None
        cv = cv_enet_gaussian(st["G"], pan, pan.xcols, ycols,
                              full_sets=[full_sets[k] for k in mine], seg_counts=seg_counts)
        return cv

    def pick(cv):
        return (cv.coef_min if lambda_rule == "min" else cv.coef_1se).reshape(
            len(mine), 2, -1).contiguous()

    def phase_fit(st):
        cv = fit(st)
        coef = pick(cv)
        return {**st, "cv": cv, "mom": dml_residual_moments(pan, coef)}

    def phase_fit_sharded(st):
        cv = fit(st)
        coef = torch.zeros((K, 2, p1), dtype=torch.float64, device=pan.device)
        if cv is not None:
            coef.index_copy_(0, const(mine, torch.int64, pan.device), pick(cv).double())
        return {**st, "cv": cv, "coef": coef}

    def phase_resid(st):
        return {**st, "mom": dml_residual_moments(pan, st["coef"])}

    def phase_final(st):
        return {**st, "res": S.dml_finalize(st["mom"], "plr")}

    cap = bool(getattr(comm, "capturable", False))

    def reduce(name, op="sum"):
        def f(st):
            (comm.all_reduce_ if op == "sum" else comm.all_reduce_max_)(st[name])
            return st
        return Collective(f, capturable=cap)     # RCCL: captured inside the step's graph

    def reduce_sym(name):
        # C01 on the upper triangles only: the fold Grams are symmetric (csrc/gram.hip writes
        # every entry once and mirrors it), so half the bytes cross the ring; the lower
        # triangle is mirrored back from the reduced upper one
        _tri_index(pan.P, pan.device)            # built here, never inside a capture

        def f(st):
            allreduce_sym_(comm, st[name])
            return st
        return Collective(f, capturable=cap)

    if exact:
        phases = [phase_gram, phase_gram_reduce]
        if dist:
            phases.append(reduce("GX"))
        phases.append(phase_from_limbs)
        if sharded:
            phases += [phase_fit_sharded, reduce("coef")]
        else:
            def phase_fit_coef(st):
                cv = fit(st)
                return {**st, "cv": cv, "coef": pick(cv).double()}
            phases.append(phase_fit_coef)
        phases.append(phase_terms)
        if dist:
            phases.append(reduce("amax", "max"))
        phases.append(phase_limbs)
        if dist:
            phases.append(reduce("limbs"))
        phases += [phase_mom_exact, phase_final]
        return phases
    phases = [phase_gram, phase_gram_reduce]
    if dist:
        phases.append(reduce_sym("G"))
    if sharded:
        phases += [phase_fit_sharded, reduce("coef"), phase_resid]
    else:
        phases.append(phase_fit)
    if dist:
        phases.append(reduce("mom"))
    phases.append(phase_final)
    return phases


def dml_crossfit_panel(pan, folds: int, lambda_rule="min", G=None, comm=None, seg_counts=None,
                       exact=False):
    """DML-PLR on a fold-segmented panel (segment k = fold k). Returns (res[2], moments[7], cv).

    comm: optional parallel.comm.Communicator — each rank holds a row shard of every
    fold; the fold Gram stack and the score moments are all-reduced (C01, C06).
    seg_counts: global rows per fold (computed with one all-reduce when omitted).
    A truncated CV fold path NaN-poisons res (ops/enet.poison_if_truncated)."""
    st = None
    for ph in dml_phases(pan, folds, lambda_rule, comm, seg_counts, G, exact=exact):
        st = ph(st)
    return st["res"], st["mom"], st.get("cv")


# ---------------------------------------------------------------- repeated cross-fitting
def micro_fold_map(K: int, s: int) -> np.ndarray:
    """Fold of each of the K*K micro-segments m = K a + b under partition s: (a + s b) mod K.
    Every partition puts K micro-segments in every fold; for prime K the partitions
    s = 0..K-1 are pairwise distinct (two of them share one micro-segment per fold pair)."""
    a, b = np.divmod(np.arange(K * K), K)
    return (a + s * b) % K


def median_aggregate(theta: torch.Tensor, se: torch.Tensor, how: str = "median"):
    """Chernozhukov et al. (2018) §3.4, Definition 3.3: theta = median of the S split
    estimates, SE^2 = median of SE_s^2 + (theta_s - theta)^2 ("mean": the means). Medians of
    an even count average the two middle values. Device tensors in, [2] out (capturable)."""
    def med(v):
        v = torch.sort(v).values
        n = v.shape[0]
        return v[n // 2] if n % 2 else 0.5 * (v[n // 2 - 1] + v[n // 2])
    if how == "mean":
        t = theta.mean()
        return torch.stack([t, torch.sqrt((se * se + (theta - t) ** 2).mean())])
    t = med(theta)
    return torch.stack([t, torch.sqrt(med(se * se + (theta - t) ** 2))])


def dml_repeated_phases(pan, folds: int, repeats: int, lambda_rule="min", comm=None,
                        seg_counts=None, aggregate="median"):
    """Repeated K-fold cross-fitting (Chernozhukov et al. 2018 §3.4): ``repeats`` = S
    distinct K-fold partitions of the rows, one DML-PLR fit per partition, median-aggregated.
    The panel holds K*K micro-segments (segment m = K a + b); partition s puts micro-segment m
    in fold (a + s b) mod K (micro_fold_map). So ONE Gram pass gives every partition's fold
    Grams: the K*K micro-Gram stack (K01, C01) is summed per partition into its K fold
    Grams (a [K, K*K] 0/1 matrix times the stack, fp64). The S partitions' CV-LASSO paths
    (K08/K09) are ONE path launch over S*K fold Grams (S * K * (K + 1) * 2 problems, each the
    bits of its own partition's solve), then each partition's residual pass runs with its
    fold coefficients spread over the micro-segments. Phases as dml_phases (SegmentedStep
    captures them: one graph at world 1);
    the result state holds "res" [2] (the aggregate) and "splits" [S, 2]. Reference:
    the split-and-average DML of /root/reference/ate_functions.R:372-389, generalised."""
    from ..utils.graphs import Collective
    K, Sn = folds, repeats
    if pan.nseg != K * K:
        raise ValueError(f"repeated cross-fitting needs K*K = {K * K} micro-segments, the panel "
                         f"has {pan.nseg}")
    if not 1 <= Sn <= K:
        raise ValueError(f"repeats must be in 1..{K} (distinct partitions of K*K micro-segments)")
    dist = comm is not None and comm.world_size > 1
    if seg_counts is None:
        seg_counts = global_seg_counts(pan, comm) if dist else np.asarray(pan.seg_nreal)
    counts = np.asarray(seg_counts, dtype=np.float64)
    dev = pan.device
    maps = [micro_fold_map(K, s) for s in range(Sn)]
    M = [const(np.eye(K)[m].T.copy(), torch.float64, dev) for m in maps]       # [K, K*K]
    fold_counts = [np.bincount(m, weights=counts, minlength=K) for m in maps]
    mi = [const(m, torch.int64, dev) for m in maps]
    full_sets = [[j for j in range(K) if j != k] for k in range(K)]
    ycols = [pan.cols["Y"], pan.cols["W"]]
    P = pan.P
    cap = bool(getattr(comm, "capturable", False))

    def phase_gram(_):
        return {"G": gram(pan, stage="tiles")}

    def phase_gram_reduce(st):
        return {"G": gram(pan, stage="reduce", out=st["G"])}

    # every partition's fold Grams as one stack of Sn * K segments; partition s's outer fold
    # k trains on segments s K + j, j != k (disjoint per partition: no shared training set)
    Mall = torch.cat(M)                                                     # [Sn K, K*K]
    sets_all = [[s * K + j for j in fs] for s in range(Sn) for fs in full_sets]
    counts_all = np.concatenate(fold_counts)

    def phase_paths(st):
        Gs = (Mall @ st["G"].view(K * K, P * P)).view(Sn * K, P, P)
        cv = cv_enet_gaussian(Gs, pan, pan.xcols, ycols, full_sets=sets_all,
                              seg_counts=counts_all)
        coef = (cv.coef_min if lambda_rule == "min" else cv.coef_1se).reshape(Sn, K, 2, -1)
        return {**st, "coef": coef}

    def phase_split(s):
        def f(st):
            coef_m = st["coef"][s].double().index_select(0, mi[s]).contiguous()
            return {**st, f"mom{s}": dml_residual_moments(pan, coef_m)}
        return f

    def phase_final(st):
        res = torch.stack([S.dml_finalize(st[f"mom{s}"], "plr") for s in range(Sn)])
        return {**st, "splits": res, "res": median_aggregate(res[:, 0], res[:, 1], aggregate)}

    def reduce(name):
        def f(st):
            comm.all_reduce_(st[name])
            return st
        return Collective(f, capturable=cap)

    def reduce_sym(name):
        _tri_index(P, dev)

        def f(st):
            allreduce_sym_(comm, st[name])
            return st
        return Collective(f, capturable=cap)

    phases = [phase_gram, phase_gram_reduce]
    if dist:
        phases.append(reduce_sym("G"))
    phases.append(phase_paths)
    for s in range(Sn):
        phases.append(phase_split(s))
        if dist:
            phases.append(reduce(f"mom{s}"))
    phases.append(phase_final)
    return phases


def dml_repeated_panel(pan, folds: int, repeats: int, lambda_rule="min", comm=None,
                       seg_counts=None, aggregate="median"):
    """Eager run of dml_repeated_phases: (aggregate [2], splits [S, 2])."""
    st = None
    for ph in dml_repeated_phases(pan, folds, repeats, lambda_rule, comm, seg_counts, aggregate):
        st = ph(st)
    return st["res"], st["splits"]


def _exact_resid(pan, coef: torch.Tensor, mode: int, sh) -> torch.Tensor:
    """Exact-mode passes of the fused bf16 residual kernel (csrc/dml.hip): mode 1 ->
    per-block max |term| [blocks * 7] fp64; mode 2 -> per-block int64 limb sums
    [blocks * 14] (returned in an fp64-typed buffer of the same bytes)."""
    K = coef.shape[0]
    dev = pan.device
    xc = const(pan.xcols, torch.int32, dev)
    segs = const(np.asarray(pan.seg_bounds[:K], dtype=np.int64), torch.int64, dev)
    nbx = 512
    part = torch.empty(K * nbx * (7 if mode == 1 else 14), dtype=torch.float64, device=dev)
    cs, bs = pan.strides()
    c = coef.double().contiguous()
    _native.call("ate_dml_resid_exact", pan.data.data_ptr(), cs, bs, xc.data_ptr(), len(pan.xcols),
                 segs.data_ptr(), K, c.data_ptr(), pan.cols["Y_hi"], pan.cols["Y_lo"],
                 pan.cols["W_hi"], pan.cols["W_lo"], pan.cols["one"], nbx, mode,
                 None if sh is None else sh.data_ptr(), part.data_ptr(),
                 torch.cuda.current_stream().cuda_stream)
    return part


def dml_residual_moments(pan, coef: torch.Tensor) -> torch.Tensor:
    """Fused held-out residual pass (csrc/dml.hip) -> 7 fp64 moments."""
    K = coef.shape[0]
    p = len(pan.xcols)
    if not pan.data.is_cuda:
        X = pan.colmajor().double()
        moms = torch.zeros(7, dtype=torch.float64)
        for k in range(K):
            r0, r1 = pan.seg_bounds[k]
            Xs = X[:, r0:r1]
            v = Xs[pan.cols["one"]] != 0
            xs = Xs[pan.xcols]
            yv, wv = Xs[pan.cols["Y"]], Xs[pan.cols["W"]]
            yr = yv - (coef[k, 0, 0] + coef[k, 0, 1:] @ xs)
            wr = wv - (coef[k, 1, 0] + coef[k, 1, 1:] @ xs)
            moms += S.dml_moments(yr[v], wr[v])
        return moms
    dev = pan.device
    xc = const(pan.xcols, torch.int32, dev)
    segs = const(np.asarray(pan.seg_bounds[:K], dtype=np.int64), torch.int64, dev)
    bf = pan.dtype == torch.bfloat16
    # bf16: 2048 rows per block; enough blocks per fold to fill 256 CUs several times
    nbx = 512 if bf else 256
    part = torch.empty(K * nbx * 7, dtype=torch.float64, device=dev)
    mom = torch.empty(7, dtype=torch.float64, device=dev)
    bf = pan.dtype == torch.bfloat16
    # binary Y/W are exact in bf16; continuous targets use the hi+lo split columns
    y0, y1 = (pan.cols["Y_hi"], pan.cols["Y_lo"]) if bf else (pan.cols["Y"], -1)
    w0, w1 = (pan.cols["W_hi"], pan.cols["W_lo"]) if bf else (pan.cols["W"], -1)
    cs, bs = pan.strides()
    _native.call("ate_dml_resid_moments", dtype_code(pan.data), pan.data.data_ptr(), cs, bs,
                 xc.data_ptr(), p, segs.data_ptr(), K, coef.data_ptr(), y0, y1, w0, w1,
                 pan.cols["one"], nbx, part.data_ptr(), mom.data_ptr(),
                 torch.cuda.current_stream().cuda_stream)
    return mom


def _dml_body(pan, folds, lambda_rule, dist=None, counts=None):
    """The whole cross-fit as one device function (GraphCache captures it: Gram, its
    all-reduce over row shards, CV-LASSO paths, selection, residual pass, the moment
    all-reduce, theta / SE = ONE graph launch)."""
    comm = dist.comm if dist is not None else None
    return dml_crossfit_panel(pan, folds, lambda_rule, comm=comm,
                              seg_counts=None if counts is None else np.asarray(counts))[0]


def _dml_graphed(pan, folds, lambda_rule, dist=None):
    """Graph-cached cross-fit keyed by the panel layout (utils/graphs.GraphCache: first
    call eager, second captures after a warm-up run, later calls copy + replay; a failed
    capture falls back to eager with the reason printed; retained HBM is bounded and
    released by utils.graphs.clear_graph_caches). ``dist`` over RCCL: the collectives
    are captured too. Returns (res, replayed)."""
    counts = None
    if dist is not None and dist.world > 1:
        counts = tuple(global_seg_counts(pan, dist.comm).tolist())   # host ints, outside
    return estimator_graphs.run("dml_plr", _dml_body, (pan,), folds, lambda_rule, dist, counts)


def _dml_repeated_body(pan, folds, repeats, lambda_rule, aggregate):
    st = None
    for ph in dml_repeated_phases(pan, folds, repeats, lambda_rule, aggregate=aggregate):
        st = ph(st)
    return torch.cat([st["res"], st["splits"].reshape(-1)])


def dml_plr_lasso_repeated(Y, W, X, folds=5, repeats=3, seed=1991, lambda_rule="min",
                           aggregate="median", method="DML cross-fit (LASSO, repeated)",
                           device=None, dtype="f64", graph=True):
    """``repeats`` = S distinct K-fold cross-fits, median-aggregated (dml_repeated_phases).
    Rows go to K*K micro-segments by a balanced Philox assignment (parallel.rng.fold_ids
    with K*K groups); partition s is micro_fold_map(K, s). On a GPU the whole call (one
    Gram pass, S path solves and residual passes, the aggregate) is one captured graph.
    Matches reference.estimators.dml_plr_lasso_repeated. diagnostics["splits"]: the S
    (ATE, SE) pairs."""
    dev = resolve_device(device)
    Yn, Wn, Xn = as_np(Y), as_np(W), as_np(X)
    micro = rng.fold_ids(len(Yn), folds * folds, seed, 0)
    pan = build_panel(Xn, Wn, Yn, folds=micro, dtype=dtype, device=dev)
    if graph and pan.data.is_cuda:
        out, g = estimator_graphs.run("dml_repeated", _dml_repeated_body, (pan,), folds, repeats,
                                      lambda_rule, aggregate)
    else:
        out, g = _dml_repeated_body(pan, folds, repeats, lambda_rule, aggregate), False
    v = out.detach().double().cpu().numpy()
    return AteResult.make(method, v[0], v[1], n=len(Yn), repeats=repeats, aggregate=aggregate,
                          splits=v[2:].reshape(repeats, 2).tolist(), hipgraph=g)


def dml_plr_lasso(Y, W, X, folds=5, seed=1991, lambda_rule="min", method="DML cross-fit (LASSO)",
                  device=None, dtype="f64", dist=None, graph=True):
    """K-fold cross-fit partially-linear DML with CV-LASSO nuisances E[Y|X], E[W|X]
    (inner CV over the other K-1 folds). Matches reference.estimators.dml_plr_lasso.

    graph: on a GPU (alone, or row-sharded over RCCL with the all-reduces captured), the
    estimator runs as one captured hipGraph (first call of a panel layout eager, captured
    on the second, replayed afterwards)."""
    dev = resolve_device(device)
    Yn, Wn, Xn = as_np(Y), as_np(W), as_np(X)
    fid = _fold_ids(len(Yn), folds, seed, 0, dist)
    pan = build_panel(Xn, Wn, Yn, folds=fid, dtype=dtype, device=dev)
    if graph and (dist is None or dist.capturable) and pan.data.is_cuda:
        res, g = _dml_graphed(pan, folds, lambda_rule, dist)
        return read_result(res, method, n=dist.n_total if dist is not None else len(Yn),
                           hipgraph=g)
    res, mom, _ = dml_crossfit_panel(pan, folds, lambda_rule,
                                     comm=dist.comm if dist is not None else None)
    return read_result(res, method, n=dist.n_total if dist is not None else len(Yn))
