"""K-fold cross-fitted AIPW with pluggable nuisance learners (BASELINE config 3:
"AIPW ATE with random-forest nuisance + 5-fold cross-fit"), and the causal-forest
ATE with a replicate-sharded bootstrap SE (config 4).

The reference's ``doubly_robust`` (ate_functions.R:149-207) fits its nuisances
in-sample (OOB forest propensity, full-data logistic outcome model) and keeps the
'+' sign quirk (Q7); this is the textbook cross-fitted version:

    for each fold k:  e_k = P(W=1|X), mu1_k = E[Y|X,W=1], mu0_k = E[Y|X,W=0]
                      trained on the other folds, predicted on fold k
    Gamma_i = mu1 - mu0 + W (Y - mu1) / e - (1 - W) (Y - mu0) / (1 - e)
    tau = mean(Gamma),  se = sd(Gamma) / sqrt(n)

Learners: ``"rf"`` (histogram forests; ``comm`` shards the trees over ranks, C05),
``"glm"`` (logistic IRLS on the device), ``"gbdt"`` (histogram gradient boosting).
"""
from __future__ import annotations

import math
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

from .. import _native
from ..models import forest as F
from ..ops.linalg import logistic, logistic_irls
from ..ops.panel import build_panel
from ..ops.scan import compact_rows
from ..parallel import rng
from ..result import AteResult
from .common import as_np, resolve_device

# format tag of the config-4 forest checkpoint key (bump when the forest outputs change)
CF_CKPT_VERSION = 2


def _backend(dev):
    return "gpu" if dev.type == "cuda" else "cpu"


def _binary(y):
    y = torch.as_tensor(y)
    return bool(torch.all((y == 0) | (y == 1)))


def _rf_fit_predict(Xb, tr_idx, ytr, ho_idx, num_trees, seed, dev, comm, edges):
    """Forest on the training columns of the binned matrix ``Xb`` [p][n] (gathered where
    it lives: no host slicing of X), predictions for the held-out columns -> tensor on
    ``dev``."""
    kind = F.KIND_CLASS if _binary(ytr) else F.KIND_REG
    p = Xb.shape[0]
    kw = dict(y=ytr) if kind == F.KIND_CLASS else dict(r1=ytr, min_node=5, mtry=max(1, p // 3))
    Xt = Xb.index_select(1, tr_idx)
    Xho = Xb.index_select(1, ho_idx)
    if comm is not None and comm.world_size > 1:
        t0, cnt = F.tree_shard(num_trees, 1, comm.rank, comm.world_size)
        fr = F.fit_forest_binned(Xt, edges, kind, ntree=cnt, seed=seed, tree_offset=t0, **kw)
        out = F.predict_tree_parallel(fr, comm, Xb=Xho, host=False)
    else:
        fr = F.fit_forest_binned(Xt, edges, kind, ntree=num_trees, seed=seed, **kw)
        out = fr.predict_binned(Xho, host=False)
    return torch.as_tensor(out, dtype=torch.float64, device=dev)


def _glm_fit_predict(Xd, tr_idx, ytr_host, ho_idx, dev):
    """Logistic IRLS on the training rows (panel assembled from the device X), fitted
    probabilities of the held-out rows on the device."""
    pan = build_panel(Xd.index_select(0, tr_idx), None, ytr_host, dtype="f64", device=dev,
                      extra_cols=("z",))
    cols = [pan.cols["one"], *pan.xcols]
    fit = logistic_irls(pan, cols, pan.cols["Y"], pan.cols["z"])
    beta = torch.nan_to_num(fit.beta.double(), nan=0.0).to(dev)
    eta = beta[0] + Xd.index_select(0, ho_idx) @ beta[1:]
    return logistic(eta)


def _gbdt_fit_predict(y, train, ho, Xb, edges, dev, seed, gbdt_kw):
    """Trees learn from ``train`` rows of the shared binned panel; the held-out
    predictions are the trainer's final scores of the ``ho`` rows (device tensors)."""
    from ..models import gbdt as G
    loss = "logistic" if _binary(y[train]) else "squared"
    be = _backend(dev)
    m = G.fit_gbdt(None, y if be == "gpu" else y.cpu().numpy(), loss=loss,
                   train=train if be == "gpu" else train.cpu().numpy(), seed=seed, backend=be,
                   edges=edges, Xb=Xb, **(gbdt_kw or {}))
    f = torch.as_tensor(m.scores, dtype=torch.float64).to(dev)[ho]
    return logistic(f) if loss == "logistic" else f


_NAMES = ("e", "mu1", "mu0")


def _agreed_flags(have, comm, dev):
    """Per-stage "already on disk" flags that every rank agrees on: the minimum over
    ranks (a stage counts as done only if every rank saved it), so tree-parallel ranks
    skip or recompute the same stages and their collectives stay paired."""
    flags = torch.tensor([float(h) for h in have], dtype=torch.float64)
    if comm is not None and comm.world_size > 1 and len(have):
        fd = flags.to(dev) if getattr(comm, "capturable", False) else flags
        comm.all_reduce_min_(fd)
        flags = fd.cpu()
    return [bool(f > 0) for f in flags]


def _panel_key(pan, data_key, *params):
    """Checkpoint key of an HBM panel run: the caller's name for the data, a content hash
    of a strided sample of the panel's rows (two panels with the same n and p but other
    data never share a key) and every parameter that changes the predictions."""
    from ..utils.checkpoint import fingerprint
    d = pan.data
    # ~4096 rows: every k-th 64-row block of a blocked panel, every k-th row otherwise
    samp = (d[::max(1, d.shape[0] // 64)] if pan.blocked else
            d[:, ::max(1, d.shape[1] // 4096)]).float().cpu().numpy()
    return f"{data_key}.{fingerprint(samp, np.asarray(params, dtype=np.float64))}"


class _JobCache:
    """Per-job checkpoint of held-out nuisance predictions: job j of a
    cross-fit (fold j // 3, nuisance _NAMES[j % 3]) saves its predictions once computed;
    a resumed run loads finished jobs instead of refitting them. Every rank decides from
    the same all-reduced flags (tree-parallel ranks must skip the same forests)."""

    def __init__(self, ck, key, tag, comm, dev, njobs):
        self.ck, self.key, self.tag = ck, key, tag
        self.done = set()
        if ck is None:
            return
        flags = _agreed_flags([ck.has(self.stage(j), key) for j in range(njobs)], comm, dev)
        self.done = {j for j in range(njobs) if flags[j]}

    def stage(self, j):
        return f"aipw_fold{j // 3}_{_NAMES[j % 3]}{self.tag}"

    def load(self, j, dev, field="pred"):
        return torch.as_tensor(self.ck.load(self.stage(j), self.key)[field], device=dev)

    def save(self, j, arr, field="pred"):
        if self.ck is not None:
            self.ck.save(self.stage(j), self.key, **{field: arr.detach().cpu().numpy()})


def aipw_score(Y, W, e, mu1, mu0, clip=0.01):
    """Textbook AIPW score on the device: Gamma = mu1 - mu0 + W (Y - mu1) / e
    - (1 - W) (Y - mu0) / (1 - e), e clipped to [clip, 1 - clip]; -> (tau, se, e)."""
    e = e.clamp(clip, 1 - clip)
    gamma = mu1 - mu0 + W * (Y - mu1) / e - (1 - W) * (Y - mu0) / (1 - e)
    n = gamma.numel()
    return gamma.mean(), gamma.std() / math.sqrt(n), e


def aipw_crossfit(Y, W, X, folds=5, learner="rf", num_trees=500, seed=1991, fold_stream=11,
                  clip=0.01, method=None, device=None, comm=None, gbdt_kw=None,
                  checkpoint=None) -> AteResult:
    """K-fold cross-fitted AIPW. X moves to ``device`` once (and is binned there for the
    tree learners); every training / held-out set is gathered on the device, every
    nuisance prediction stays there, and the score, its mean and SE are computed on the
    device (one read-back of the result). ``checkpoint`` (utils/checkpoint.Checkpoint):
    finished (fold, nuisance) predictions are saved and reloaded on a rerun."""
    dev = resolve_device(device)
    Yn, Wn, Xn = as_np(Y), as_np(W), as_np(X)
    n = len(Yn)
    fid = torch.as_tensor(rng.fold_ids(n, folds, seed, fold_stream), device=dev)
    Yd = torch.as_tensor(Yn, dtype=torch.float64, device=dev)
    Wd = torch.as_tensor(Wn, dtype=torch.float64, device=dev)
    e = torch.empty(n, dtype=torch.float64, device=dev)
    mu1 = torch.empty_like(e)
    mu0 = torch.empty_like(e)
    Xd = Xb = edges = None
    if learner == "rf":
        edges = F.bin_edges(Xn)
        Xb = F.bin_matrix(Xn, edges[0], edges[1], dev if dev.type == "cuda" else None)
    elif learner == "gbdt":
        from ..models import gbdt as G
        edges = G.sample_bin_edges(Xn, device=dev)
        Xb = G.binned(Xn, edges, dev)
    elif learner == "glm":
        Xd = torch.as_tensor(Xn, dtype=torch.float64, device=dev)
    else:
        raise ValueError(learner)
    key = ""
    if checkpoint is not None:
        from ..utils.checkpoint import fingerprint
        key = fingerprint(Yn, Wn, Xn, np.array([folds, num_trees, seed, fold_stream]),
                          np.frombuffer(learner.encode(), dtype=np.uint8),
                          np.frombuffer(repr(sorted((gbdt_kw or {}).items())).encode(),
                                        dtype=np.uint8))
    tag = "" if comm is None or comm.world_size == 1 else f".r{comm.rank}of{comm.world_size}"
    cache = _JobCache(checkpoint, key, tag, comm, dev, 3 * folds)
    jobs = []
    # row lists by a lookback-free compaction on this stream, before the jobs run side by
    # side on their own streams (ops/scan.py: torch.nonzero there stalled config 3)
    for k in range(folds):
        ho = fid == k
        tr = ~ho
        t1, t0 = tr & (Wd == 1), tr & (Wd == 0)
        sd = seed + 1000 * (k + 1)
        hoi = compact_rows(ho)
        rl = (lambda m: compact_rows(m)) if learner in ("rf", "glm") else (lambda m: None)
        jobs += [(e, ho, tr, Wd, sd, 3 * k, hoi, rl(tr)),
                 (mu1, ho, t1, Yd, sd + 1, 3 * k + 1, hoi, rl(t1)),
                 (mu0, ho, t0, Yd, sd + 2, 3 * k + 2, hoi, rl(t0))]

    def run(job):
        out, ho, rows, target, sd, j, hoi, ri = job
        if j in cache.done:
            out.index_copy_(0, hoi, cache.load(j, dev))
            return
        if learner == "rf":
            r = _rf_fit_predict(Xb, ri, target.index_select(0, ri), hoi, num_trees, sd, dev,
                                comm, edges)
        elif learner == "glm":
            r = _glm_fit_predict(Xd, ri, target.index_select(0, ri).cpu().numpy(), hoi, dev)
        else:
            r = _gbdt_fit_predict(target, rows, ho, Xb, edges, dev, sd, gbdt_kw)
        out.index_copy_(0, hoi, r)
        cache.save(j, r)

    concurrent = learner == "rf" and dev.type == "cuda" and (comm is None or comm.world_size == 1)
    if concurrent:
        # the 3K forests are independent: grow them concurrently, one HIP stream per host
        # thread, so a 100-tree forest (100 workgroups) does not leave most CUs idle;
        # every forest is a deterministic function of its inputs (same trees as serially)
        main = torch.cuda.current_stream(dev)

        def run_on(job):
            st = torch.cuda.Stream(device=dev)
            st.wait_stream(main)
            with torch.cuda.device(dev), torch.cuda.stream(st):
                run(job)
            st.synchronize()

        with ThreadPoolExecutor(max_workers=min(len(jobs), 8)) as ex:
            list(ex.map(run_on, jobs))
    else:
        for job in jobs:
            run(job)
    tau, se, ec = aipw_score(Yd, Wd, e, mu1, mu0, clip)
    v = torch.stack([tau, se, ec.min(), ec.max()]).cpu().numpy()
    return AteResult.make(method or f"AIPW cross-fit ({learner}, K={folds})", float(v[0]),
                          float(v[1]), e_min=float(v[2]), e_max=float(v[3]), device_scores=True)


def aipw_rf_crossfit_panel(pan, num_trees=100, seed=1991, clip=0.01, comm=None,
                           tree_shard=None, concurrent=True, engine="gpu",
                           method="AIPW cross-fit (rf, HBM panel)", checkpoint=None,
                           data_key="") -> AteResult:
    """Config 3 on an HBM-resident panel (data/device_dgp.synthetic_panel, segment k =
    fold k): the panel's feature columns are binned on the device (``bin_panel``, no host
    copy of X) into the forest engine's column-major uint8 layout; per fold, the
    propensity forest (W on the other folds) and the two outcome forests (Y on the other
    folds' treated / control rows) are grown from device-gathered training columns and
    predict the held-out fold's bins; the AIPW scores and their mean / sd are computed in
    fp64 on the device.

    Trees are sharded over ``comm`` (one rank per GPU, every rank holding all binned rows
    and growing its share of every forest), or over a simulated ``tree_shard=(rank,
    world)`` on one device (the per-GPU work of a multi-GPU run; the ATE is then that of
    the shard's trees). At every world size each forest leaves only its LOCAL held-out vote
    sums (prediction phase 1, csrc/forest.hip); after all 3K forests, the sums of every
    job are packed into ONE buffer and all-reduced once (C05), then divided by the tree
    counts (= forest_final_kernel). Votes are integers, so the predictions -- and the ATE
    and SE -- are the same bits at every world size. ``concurrent``: the 3K forests grow
    side by side on separate streams, in batches that fit free HBM (a forest of T trees
    fills only T CUs), at every world size.
    ``engine="cpu"`` grows the same forests on the host engine from the same bins
    (bit-identical trees; the parity test). ``checkpoint`` (+ ``data_key``, a name of the
    panel's data; a sample of the panel is hashed too): each job's local vote sums are
    saved per rank; a rerun loads them and grows only the missing forests."""
    from .boosting import bin_panel
    dev = pan.device
    K = pan.nseg
    Xr, ldr, edges, rows = bin_panel(pan)
    p = len(pan.xcols)
    Xb = Xr[:, :p].t().contiguous()                  # [p][n] engine layout
    del Xr
    nr = np.asarray(pan.seg_nreal, dtype=np.int64)
    c0 = np.concatenate([[0], np.cumsum(nr)]).astype(np.int64)
    n = int(c0[-1])
    Y = pan.col("Y").index_select(0, rows).double()
    W = pan.col("W").index_select(0, rows).double()
    if comm is not None and comm.world_size > 1:
        rank, world = comm.rank, comm.world_size
    elif tree_shard is not None:
        rank, world = tree_shard
    else:
        rank, world = 0, 1
    t0, cnt = F.tree_shard(num_trees, 1, rank, world)
    pcomm = comm if comm is not None and comm.world_size > 1 else None
    ar = torch.arange(n, device=dev)
    tag = "" if pcomm is None else f".r{rank}of{world}"
    key = _panel_key(pan, data_key, n, p, num_trees, seed, t0, cnt) \
        if checkpoint is not None else ""
    cache = _JobCache(checkpoint, key, tag, pcomm, dev, 3 * K)
    # job j = 3k + {0: e (W on the other folds), 1: mu1 (Y, treated), 2: mu0 (Y, control)};
    # its local sums live at pack[off_j : off_j + 2 nho_k] (votes, then trees counted)
    off = np.concatenate([[0], np.cumsum([2 * int(nr[j // 3]) for j in range(3 * K)])])
    pack = torch.zeros(int(off[-1]), dtype=torch.int64, device=dev)   # fixed-point sums
    jobs = []
    for k in range(K):
        a, b = int(c0[k]), int(c0[k + 1])
        tr = (ar < a) | (ar >= b)
        sd = seed + 1000 * (k + 1)
        for j, (mask, target, s_) in enumerate(((tr, W, sd), (tr & (W == 1), Y, sd + 1),
                                               (tr & (W == 0), Y, sd + 2))):
            jobs.append((mask, target, s_, a, b, 3 * k + j))
    todo = []
    for jb in jobs:                          # finished jobs of an earlier run: their sums
        j = jb[-1]
        if j in cache.done:
            pack[off[j]:off[j + 1]] = cache.load(j, dev, "sums")
        else:
            todo.append(jb)
    # training rows of every job, computed here on the caller's stream: a lookback-free
    # compaction (ops/scan.py) and never inside the side-by-side forests below, where
    # torch.nonzero's spinning workgroups stalled the shard (profiles/r03_cfg3b)
    jobs = [(compact_rows(mask), target, sd, a, b, j) for mask, target, sd, a, b, j in todo]

    def run(job):
        idx, target, sd, a, b, j = job
        yt = target.index_select(0, idx)
        binary = bool(((yt == 0) | (yt == 1)).all())
        kw = dict(y=yt) if binary else dict(r1=yt, min_node=5, mtry=max(1, p // 3))
        Xt = Xb.index_select(1, idx)
        if engine == "cpu":
            Xt = Xt.cpu().numpy()
        fr = F.fit_forest_binned(Xt, edges, F.KIND_CLASS if binary else F.KIND_REG,
                                 ntree=cnt, seed=sd, tree_offset=t0, **kw)
        del Xt
        Xho = Xb[:, a:b].contiguous()
        if fr.backend == "cpu":
            Xho = Xho.cpu().numpy()
        st = fr.new_state(b - a)
        fr.predict_state(Xho, False, st, phases=1)          # this rank's trees only
        loc = torch.as_tensor(st[:2 * (b - a)], device=dev)
        pack[off[j]:off[j + 1]] = loc
        cache.save(j, loc, "sums")

    if concurrent and dev.type == "cuda" and engine == "gpu" and len(jobs) > 1:
        # the 3K forests are independent: grow them side by side (one stream per host
        # thread; a forest of T trees fills only T CUs), in batches whose working set
        # (training bins + node arrays + growth scratch) fits a share of free HBM
        free = torch.cuda.mem_get_info(dev)[0]
        lib = _native.hip()

        def need(job):
            nt = job[0].numel()
            base = p * nt + cnt * (2 * nt + 1) * 20 + cnt * nt      # bins, trees, in-bag
            if F.LEVEL_MIN_ROWS <= nt:
                # level engine: row-major copy, weights / positions, level lists
                return base + p * nt + cnt * nt * 12 + cnt * nt * 56
            return base + int(lib.ate_forest_scratch_bytes(nt, cnt))

        # forests on the level engine fill the GPU by themselves: a few side by side only
        # hide each other's per-level host syncs (ATE_CF_CONCURRENT caps the batch;
        # profiles/r03_cfg3: 1 -> 10.3 s, 2 -> 9.4, 3 -> 8.7, 5 -> 8.4 for the config-3
        # per-GPU shard; r03_cfg3b, lookback-free scans: 3 -> 8.0 s, 5 -> 7.7 s)
        cap_b = int(os.environ.get("ATE_CF_CONCURRENT", "5")) or len(jobs)
        batches, cur_b, used = [], [], 0
        for job in jobs:
            m = need(job)
            if cur_b and (used + m > 0.6 * free or len(cur_b) >= cap_b):
                batches.append(cur_b)
                cur_b, used = [], 0
            cur_b.append(job)
            used += m
        batches.append(cur_b)
        main = torch.cuda.current_stream(dev)

        def run_on(job):
            st = torch.cuda.Stream(device=dev)
            st.wait_stream(main)
            with torch.cuda.device(dev), torch.cuda.stream(st):
                run(job)
            st.synchronize()

        for bt in batches:
            with ThreadPoolExecutor(max_workers=len(bt)) as ex:
                list(ex.map(run_on, bt))
    else:
        for job in jobs:
            run(job)
    if pcomm is not None:
        pcomm.all_reduce_(pack)              # C05: every job's vote sums, one collective
    e = torch.empty(n, dtype=torch.float64, device=dev)
    mu1 = torch.empty_like(e)
    mu0 = torch.empty_like(e)
    for j in range(3 * K):
        k = j // 3
        a, b = int(c0[k]), int(c0[k + 1])
        s_ = pack[off[j]:off[j + 1]]
        votes = s_[:b - a].double() / F.FIX           # from_fix: 2^-32 fixed point
        used = s_[b - a:].double()
        # forest_final_kernel: votes / trees (NaN for a row no tree reached)
        (e, mu1, mu0)[j % 3][a:b] = torch.where(used > 0, votes / used,
                                                torch.full_like(votes, float("nan")))
    tau, se, ec = aipw_score(Y, W, e, mu1, mu0, clip)
    v = torch.stack([tau, se, ec.min(), ec.max()]).cpu().numpy()
    return AteResult.make(method, float(v[0]), float(v[1]), n=n, trees=num_trees,
                          trees_this_device=cnt, e_min=float(v[2]), e_max=float(v[3]))


def causal_forest_bootstrap(Y, W, X, num_trees=2000, B=1000, seed=12345, boot_seed=1991,
                            method="Causal Forest(GRF) + bootstrap SE", device=None, comm=None,
                            nuisance_trees=None, checkpoint=None, boot_chunk=250,
                            compat="reference") -> AteResult:
    """Config 4: grf-style causal forest (trees sharded over ``comm``), AIPW scores
    Gamma_i from the OOB CATEs, and B multinomial bootstrap replicates of mean(Gamma)
    sharded over the ranks (C07); SE = sd of the replicates. The scores are formed and
    resampled on the device. ``checkpoint``: the forest outputs and every range of
    ``boot_chunk`` replicates are saved once computed; a rerun resumes from them with
    identical results (every draw is keyed by (seed, replicate, row))."""
    from .linear import bootstrap_replicates
    dev = resolve_device(device)
    Xn, Yn, Wn = as_np(X), as_np(Y), as_np(W)
    key, tag = "", ""
    if checkpoint is not None:
        from ..utils.checkpoint import fingerprint
        # everything that changes the forest outputs: the resolved split engine, the
        # orthogonalisation forests' little-bag size, the causal split rule and a format tag
        # (an older checkpoint of binned / group-2 / unbalanced-split forests must not load)
        sp = F.resolve_splits("auto", len(Yn), Xn.shape[1])
        key = fingerprint(Yn, Wn, Xn, np.array([num_trees, seed, nuisance_trees or 0]),
                          np.frombuffer(f"v{CF_CKPT_VERSION}|{sp}|ng1|{F.CAUSAL_SPLIT_RULE}"
                                        .encode(), dtype=np.uint8))
        tag = "" if comm is None or comm.world_size == 1 else f".r{comm.rank}of{comm.world_size}"
    stage = f"cf_fit{tag}"
    ranges = [(b0, min(boot_chunk, B - b0)) for b0 in range(0, B, boot_chunk)]
    bkey = key + f".{boot_seed}"
    have = [False] * (1 + len(ranges))
    if checkpoint is not None:
        # every rank must skip / recompute the same stages: causal_forest (tree-sharded
        # collectives) and bootstrap_replicates (all-gather) pair up across ranks
        have = _agreed_flags([checkpoint.has(stage, key)] +
                             [checkpoint.has(f"cf_boot_{b0}_{b0 + nb}{tag}", bkey)
                              for b0, nb in ranges], comm, dev)
    if have[0]:
        z = checkpoint.load(stage, key)
        y_hat, w_hat, tau_oob = z["y_hat"], z["w_hat"], z["tau_oob"]
    else:
        cf = F.causal_forest(Xn, Yn, Wn, num_trees=num_trees, seed=seed,
                             nuisance_trees=nuisance_trees, backend=_backend(dev), comm=comm)
        y_hat, w_hat, tau_oob = cf.y_hat, cf.w_hat, cf.tau_oob
        if checkpoint is not None:
            checkpoint.save(stage, key, y_hat=y_hat, w_hat=w_hat, tau_oob=tau_oob,
                            var_oob=cf.var_oob)
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=dev)
    Yd, Wd, yh, wh, to = t(Yn), t(Wn), t(y_hat), t(w_hat), t(tau_oob)
    w_res = Wd - wh
    tau = torch.where(torch.isnan(to), torch.nanmean(to), to)
    # grf's AIPW does not clip W.hat (compat="reference"; a poor-overlap warning as grf);
    # compat="textbook" clips it to [1e-6, 1 - 1e-6]
    F.overlap_warning(float(wh.min()), float(wh.max()))
    what = wh if compat == "reference" else wh.clamp(F.AIPW_TEXTBOOK_CLIP,
                                                     1 - F.AIPW_TEXTBOOK_CLIP)
    g = tau + w_res / (what * (1 - what)) * (Yd - yh - tau * w_res)
    n = g.numel()
    est, se_aipw = g.mean(), g.std() / math.sqrt(n)      # models/forest.average_treatment_effect
    zeros = torch.zeros_like(g)
    parts = []
    for i, (b0, nb) in enumerate(ranges):
        bst = f"cf_boot_{b0}_{b0 + nb}{tag}"
        if have[1 + i]:
            parts.append(t(checkpoint.load(bst, bkey)["taus"]))
            continue
        tb = bootstrap_replicates(g, zeros, nb, boot_seed, comm, b_start=b0)
        if checkpoint is not None:
            checkpoint.save(bst, bkey, taus=tb.cpu().numpy())
        parts.append(tb.to(dev))
    taus = torch.cat(parts)
    v = torch.stack([est, taus.std(unbiased=True), se_aipw]).cpu().numpy()
    return AteResult.make(method, float(v[0]), float(v[1]), se_aipw=float(v[2]), B=B)
