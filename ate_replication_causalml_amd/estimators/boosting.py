"""DML-PLR with histogram-GBDT nuisances (BASELINE config 5: "N=1e8 p=2000 DML with
histogram-GBDT nuisance, full panel resident in 8x288 GB HBM").

For each of K folds, E[Y|X] and E[W|X] are boosted on the other folds (``train``
mask over the resident binned panel — no row copies) and predicted on fold k; the
held-out residuals feed the Neyman-orthogonal PLR score (same finalisation as the
LASSO cross-fit, ops/stats.py). The DML ancestor is ``double_ml``
(ate_functions.R:372-389), scaled to BASELINE config 5.

Row sharding (``dist``, one rank per GPU): every rank holds its rows of every fold in
HBM; bin edges come from the global strided row sample (all-gathered, so they equal the
single-device edges), each level's compact node histograms are all-reduced (C04,
exact int64) on the fit's stream, the base score is an exact fixed-point mean, and the
score moments are exact sums (ops/exact.py) all-reduced (C06). The trees, the
held-out predictions and the ATE / SE are therefore the same bits at every world size.
Y, W, the scores and the residuals stay on the device.

``checkpoint`` (utils/checkpoint.Checkpoint): the held-out predictions of every finished
fold are saved (per rank); a rerun loads them and fits only the missing folds, with
bitwise-identical results.
"""
from __future__ import annotations

import numpy as np
import torch

from ..models import gbdt as G
from ..ops import stats as S
from ..ops.linalg import logistic
from ..parallel import rng
from .common import as_np, read_result, resolve_device


def _loss(v, dist=None):
    """'logistic' for a 0/1 target (on every rank), else 'squared'."""
    t = torch.as_tensor(v)
    flag = torch.tensor([float(bool(torch.all((t == 0) | (t == 1))))], dtype=torch.float64,
                        device=t.device)
    if dist is not None:
        dist.min_(flag)
    return "logistic" if bool(flag.item()) else "squared"


def _response(m, dev):
    """Raw boosting scores of every row -> response on ``dev`` (no host copy for GPU fits)."""
    f = m.scores if isinstance(m.scores, torch.Tensor) else torch.from_numpy(np.asarray(m.scores))
    f = f.to(dev, torch.float64)
    return logistic(f) if m.loss == "logistic" else f


def _all_ranks_have(ck, stage, dkey, dist, dev):
    ok = torch.tensor([float(ck.has(stage, dkey))], dtype=torch.float64,
                      device=dev if dist is not None and getattr(dist.comm, "capturable", False)
                      else "cpu")
    if dist is not None:
        dist.min_(ok)
    return bool(ok.item())


def _pair_dist(dist):
    """The context of the second of two concurrently running fits: its own communicator
    (``dup``), or None when collectives cannot be duplicated (then the fits run serially)."""
    if dist is None or dist.world == 1:
        return dist
    dup = getattr(dist.comm, "dup", None)
    if dup is None:
        return None
    # created once per communicator and cached on it: dup() is a new process group (a
    # collective every rank runs in the same order), never re-made per cross-fit call
    second = getattr(dist.comm, "_pair_dup", None)
    if second is None:
        second = dup()
        try:
            dist.comm._pair_dup = second
        except AttributeError:      # a communicator type without instance attributes
            pass
    from ..parallel.dist import DistContext
    return DistContext(second, dist.row_offset, dist.n_total)


def _fit_pair(fit, jobs, dev, dists):
    """Run ``fit(target, loss, train, dist)`` for the two jobs of a fold side by side, each on
    its own HIP stream (the models are independent: E[Y|X] and E[W|X] on the same rows; a
    level's histogram of one overlaps the other's small deep levels and host stepping).
    Same trees as serially. ``dists``: one context per job (own communicators)."""
    from concurrent.futures import ThreadPoolExecutor
    main = torch.cuda.current_stream(dev)

    def run(i):
        st = torch.cuda.Stream(device=dev)
        st.wait_stream(main)
        with torch.cuda.device(dev), torch.cuda.stream(st):
            out = fit(*jobs[i], dists[i])
        main.wait_stream(st)
        st.synchronize()
        return out
    with ThreadPoolExecutor(max_workers=2) as ex:
        return list(ex.map(run, range(2)))


def _pair_fitter(kw):
    """fit_pair for _crossfit on the GPU: models/gbdt.fit_gbdt_pair with the fits' settings
    (None when ATE_GBDT_FUSED_ROOT=0: the two fits of a fold run one after the other)."""
    if not G.FUSED_ROOT:
        return None
    opts = {k: kw[k] for k in ("n_trees", "depth", "lr", "lam", "min_child")}

    def fit_pair(jobs, d):
        (ty, ly, tr), (tw, lw, _) = jobs
        return G.fit_gbdt_pair([ty, tw], [ly, lw], tr, kw["Xb"], kw["edges"], dist=d, **opts)
    return fit_pair


def _crossfit(y, w, fid, K, fit, dev, dist, checkpoint, dkey, concurrent=False, fit_pair=None):
    """Held-out predictions of E[Y|X], E[W|X] for every fold (device tensors). ``fit(target,
    loss, train, dist)``. ``fit_pair(jobs, dist)`` (GPU, models/gbdt.fit_gbdt_pair): a fold's
    two fits in lockstep with one fused root-histogram pass per tree pair (the same trees).
    ``concurrent`` (GPU): a fold's two fits run side by side on two
    streams, the second with a duplicated communicator -- the same bits, but slower on the
    config-5 shard (1.31 vs 1.18 s for 20 trees: the histogram kernels fill the GPU alone and
    two of them contend for L2; profiles/r04_cfg5), so off by default."""
    ey = torch.zeros_like(y)
    ew = torch.zeros_like(w)
    ly, lw = _loss(y, dist), _loss(w, dist)
    tag = "" if dist is None else f".r{dist.rank}of{dist.world}"
    d2 = _pair_dist(dist) if (concurrent and dev.type == "cuda") else None
    pair = concurrent and dev.type == "cuda" and (dist is None or d2 is not None)
    for k in range(K):
        ho = fid == k
        stage = f"dml_gbdt_fold{k}{tag}"
        if checkpoint is not None and _all_ranks_have(checkpoint, stage, dkey, dist, dev):
            z = checkpoint.load(stage, dkey)
            py = torch.as_tensor(z["ey"], device=dev)
            pw = torch.as_tensor(z["ew"], device=dev)
        else:
            # held-out predictions = the trainer's running scores of the rows it skipped
            if pair:
                my, mw = _fit_pair(fit, [(y, ly, ~ho), (w, lw, ~ho)], dev, [dist, d2])
            elif fit_pair is not None:
                my, mw = fit_pair([(y, ly, ~ho), (w, lw, ~ho)], dist)
            else:
                my, mw = fit(y, ly, ~ho, dist), fit(w, lw, ~ho, dist)
            py = torch.where(ho, _response(my, dev), torch.zeros_like(y))
            pw = torch.where(ho, _response(mw, dev), torch.zeros_like(w))
            if checkpoint is not None:
                checkpoint.save(stage, dkey, ey=py.cpu().numpy(), ew=pw.cpu().numpy())
        ey = torch.where(ho, py, ey)
        ew = torch.where(ho, pw, ew)
    return ey, ew


def dml_plr_gbdt(Y, W, X, folds=5, n_trees=100, depth=6, lr=0.1, lam=1.0, min_child=1.0,
                 seed=1991, fold_stream=0, method="DML cross-fit (GBDT)", device=None,
                 dist=None, checkpoint=None):
    """Host-array entry point: (Y, W, X) are this rank's rows (``dist``) or all rows."""
    dev = resolve_device(device)
    Yn, Wn, Xn = as_np(Y), as_np(W), as_np(X)
    n = len(Yn)
    fid = dist.fold_ids(folds, seed, fold_stream) if dist is not None else \
        rng.fold_ids(n, folds, seed, fold_stream)
    backend = "gpu" if dev.type == "cuda" else "cpu"
    edges = G.global_bin_edges(Xn, dist, device=dev)
    Xb = G.binned(Xn, edges, dev)          # binned once, shared by all 2K fits
    kw = dict(n_trees=n_trees, depth=depth, lr=lr, lam=lam, min_child=min_child,
              backend=backend, edges=edges, Xb=Xb)
    y = torch.as_tensor(Yn, dtype=torch.float64, device=dev)
    w = torch.as_tensor(Wn, dtype=torch.float64, device=dev)
    fid_t = torch.as_tensor(fid, device=dev)

    def fit(target, loss, train, d):
        tr = train if backend == "gpu" else train.cpu().numpy()
        tg = target if backend == "gpu" else target.cpu().numpy()
        return G.fit_gbdt(None, tg, loss=loss, train=tr, dist=d, **kw)

    dkey = _data_key(checkpoint, Yn, Wn, Xn, np.array([folds, n_trees, depth, lr, lam,
                                                       min_child, seed, fold_stream], float))
    ey, ew = _crossfit(y, w, fid_t, folds, fit, dev, dist, checkpoint, dkey,
                       fit_pair=_pair_fitter(kw) if backend == "gpu" else None)
    mom = S.dml_moments_exact(y - ey, w - ew, dist)
    return read_result(S.dml_finalize(mom, "plr"), method,
                       n=dist.n_total if dist is not None else n)


def _data_key(checkpoint, *arrays):
    if checkpoint is None:
        return ""
    from ..utils.checkpoint import fingerprint
    return fingerprint(*arrays)


def panel_bin_edges(pan, rows, dist=None, edge_rows=G.EDGE_SAMPLE):
    """Bin edges of the panel's feature columns from the GLOBAL strided row sample
    (models/gbdt.global_sample_ids over global row ids ``pan.row_index``): each rank
    takes its rows of the sample on the device, the pieces are all-gathered and the
    edges computed on the device (models/forest.bin_edges_device: per-column sort, so the
    edges depend on the sample's values only, not on which rank held them)."""
    from ..models import forest as F
    dev = pan.device
    n_total = dist.n_total if dist is not None else pan.n
    ids = torch.as_tensor(G.global_sample_ids(n_total, edge_rows), device=dev)
    gid = pan.row_index.index_select(0, rows)
    pick = rows[torch.isin(gid, ids)]
    xc = torch.as_tensor(pan.xcols, dtype=torch.long, device=dev)
    Xcol = pan.colmajor()
    samp = Xcol.index_select(0, xc).index_select(1, pick).t().double()        # [m, p]
    if dist is not None and dist.world > 1:
        cnt = torch.tensor([samp.shape[0]], dtype=torch.float64)
        on_dev = bool(getattr(dist.comm, "capturable", False))
        cdev = dev if on_dev else "cpu"
        counts = [int(c.item()) for c in dist.comm.all_gather(cnt.to(cdev))]
        buf = torch.zeros((max(counts), samp.shape[1]), dtype=torch.float64, device=cdev)
        buf[:samp.shape[0]] = samp.to(cdev)
        parts = dist.comm.all_gather(buf)
        samp = torch.cat([pp[:c] for pp, c in zip(parts, counts)]).to(dev)
    return F.bin_edges_device(samp) if dev.type == "cuda" else F.bin_edges(samp.numpy())


def bin_panel(pan, edges=None, edge_rows=G.EDGE_SAMPLE, dist=None):
    """Row-major uint8 bins [n_real][ldr] of the panel's feature columns, binned on the
    device (csrc/gbdt.hip gbdt_bin_panel_kernel; no host copy of X). Edges default to
    ``panel_bin_edges`` (global strided row sample). Returns (Xr, ldr, edges, rows) with
    ``rows`` the panel row of each compact row."""
    from .. import _native
    dev = pan.device
    X = pan.data
    p = len(pan.xcols)
    r0 = np.asarray(pan.seg_bounds[:, 0], dtype=np.int64)
    nr = np.asarray(pan.seg_nreal, dtype=np.int64)
    c0 = np.concatenate([[0], np.cumsum(nr)[:-1]]).astype(np.int64)
    n = int(nr.sum())
    rows = torch.cat([torch.arange(int(a), int(a + m), device=dev) for a, m in zip(r0, nr)])
    if edges is None:
        edges = panel_bin_edges(pan, rows, dist, edge_rows)
    ldr = -(-p // 32) * 32
    Xr = torch.zeros((n, ldr), dtype=torch.uint8, device=dev)
    if dev.type != "cuda":
        # host twin of gbdt_bin_panel_kernel: bin(x) = #{edges < x} (lower bound)
        Xc = pan.colmajor()
        for j, c in enumerate(pan.xcols):
            e = torch.as_tensor(edges[0][j, :int(edges[1][j])], dtype=torch.float64)
            Xr[:, j] = torch.searchsorted(e, Xc[c].index_select(0, rows).double().contiguous(),
                                          right=False).to(torch.uint8)
        return Xr, ldr, edges, rows
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
                       method="DML cross-fit (GBDT)", dist=None, checkpoint=None,
                       data_key="", edge_rows=G.EDGE_SAMPLE, concurrent=False):
    """Config 5 on an HBM-resident panel (data/device_dgp.synthetic_panel, segment k =
    fold k; with ``dist`` this rank's slice of every fold): device binning from the global
    edge sample, then the K-fold cross-fit on the resident row-major bins with Y, W,
    scores and residuals on the device; histograms (C04) and moments (C06) all-reduced.
    ``checkpoint`` + ``data_key`` (a caller-chosen name of the data, e.g. the synthetic
    panel's (n, p, seed)): per-fold held-out predictions are saved / resumed."""
    dev = pan.device
    if dev.type != "cuda":
        raise ValueError("dml_plr_gbdt_panel runs on a GPU panel (use dml_plr_gbdt on host arrays)")
    Xr, ldr, edges, rows = bin_panel(pan, edge_rows=edge_rows, dist=dist)
    K = pan.nseg
    nr = torch.as_tensor(np.asarray(pan.seg_nreal, dtype=np.int64), device=dev)
    y = pan.col("Y").index_select(0, rows).double()
    w = pan.col("W").index_select(0, rows).double()
    fid = torch.repeat_interleave(torch.arange(K, device=dev), nr)
    kw = dict(n_trees=n_trees, depth=depth, lr=lr, lam=lam, min_child=min_child,
              backend="gpu", edges=edges, Xb=(Xr, ldr))

    def fit(target, loss, train, d):
        return G.fit_gbdt(None, target, loss=loss, train=train, dist=d, **kw)

    dkey = ""
    if checkpoint is not None:
        from .crossfit import _panel_key
        dkey = _panel_key(pan, data_key, pan.n, len(pan.xcols), n_trees, depth, lr, lam,
                          min_child, edge_rows)
    ey, ew = _crossfit(y, w, fid, K, fit, dev, dist, checkpoint, dkey, concurrent,
                       fit_pair=_pair_fitter(kw))
    mom = S.dml_moments_exact(y - ey, w - ew, dist)
    n_all = dist.n_total if dist is not None else pan.n
    return read_result(S.dml_finalize(mom, "plr"), method, n=n_all, trees=n_trees, depth=depth)
