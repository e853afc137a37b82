#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): rows/sec of the K-fold cross-fit DML-ATE
(partially linear model, CV-LASSO nuisances for E[Y|X] and E[W|X]) at N=1e7,
p=500 on 1/2/4/8 MI355X.

One "step" = one complete ``ate_dml`` call on the HBM-resident bf16 panel:
per-fold MFMA Gram stack (K01) -> RCCL all-reduce of the Gram stack (C01) ->
for each of the 5 outer folds and both nuisances: glmnet-equivalent LASSO path
(100 lambdas) + 4-fold inner CV + lambda.min selection on device (K08/K09) ->
fused held-out residual pass + orthogonal-score moments (csrc/dml.hip) ->
all-reduce of the moments (C06) -> theta / SE on device.
Nothing is cached across steps; every nuisance is refit each step.

Data (``--dgp``, default ``tutorial``): the tutorial's selection-biased ``df_mod`` at
scale (data/device_dgp.py, data/panel_selection.py): the calibrated
latent-voter model drawn as an RCT, then ``ate_replication.Rmd:97-121``'s transform over
the generated rows (the first round(0.85 k) treated likely voters and control unlikely
voters dropped), N = 1e7 rows KEPT per GPU (``n_generated`` in the JSON: ~5.5e7 drawn),
21 tutorial covariates + 479 extra nuisance covariates, generated directly in HBM
(random-init equivalent: there is no dataset download). W is confounded with the vote
history there. ``--also-rct 1`` (default) then measures the same step on the RCT panel
(``--dgp rct``: W independent of X, every coordinate of the W path moves -- the path
solver's worst case) and reports it under ``"rct"``.

Timed step (the metric of record): ONE ``ate_dml`` call on the resident
panel, captured as the library runs it (one stream, the default Gram plan). The K timed
steps are K such calls back to back on one stream; stream order serialises them, so no
two fits overlap. ``value`` = N / ms_per_step. ``single_fit_ms`` is the median of >= 5
replays each bracketed by device syncs (the §7.5 latency). The panel uses the 64-row
blocked layout (``--blocked 1``) with its 128 exactly-{0,1} columns also stored as bytes
(``layout`` "blocked64+bytes8": the Gram reads 896 instead of 1,024 bytes per row, the
same bits; data/device_dgp.py). With RCCL the all-reduces (C01 Gram stack, C08
coefficients, C06 moments) are captured inside the call's graph
(utils/graphs.SegmentedStep); if capture of the collectives fails they run eagerly between
graph segments and the JSON says so (``collectives_captured``).

Secondary, reported under ``throughput_inflight`` and never as ``value``: ``--inflight 3``
identical calls overlapped on streams (each fit's Gram on one low-priority stream beside
another fit's latency-bound path solve), with a check that they return the same bits.
Secondary, under ``repeated`` (world 1, ``--repeats 3``): ``ate_dml(repeats=3)``, three
DISTINCT 5-fold partitions of 25 micro-segments from one Gram pass and one path launch,
median-aggregated (Chernozhukov et al. 2018 §3.4); the JSON lists the split ATEs.

Parity (``--parity 1``, untimed): the same kept rows as a float64 panel, fp64 Gram and
fp64 path solves; the JSON reports |dATE| / SE_f64 and the relative SE difference.

Scaling: weak by default (N=1e7 rows per GPU; at N=1 GPU this is exactly the
BASELINE config); ``--scaling strong`` keeps N=1e7 in total.

    python bench.py --gpus N --steps K --warmup W
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)
"""
from __future__ import annotations

import argparse
import contextlib
import json
import math
import os
import sys
import time


# BASELINE.md "Measured CPU comparison point": the reference publishes no throughput; the
# conservative CPU bound is the fp32 fold-Gram stack alone on the 8-core host
# (tools/cpu_baseline.py -> profiles/r02_cpu_baseline.json), rows/s at N=1e7, p=500.
CPU_BASELINE_ROWS_PER_S = 1.154e6


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=float, default=1e7,
                    help="rows per GPU (weak scaling) or in total (strong scaling); with "
                         "--dgp tutorial these are rows KEPT by the selection transform")
    ap.add_argument("--p", type=int, default=500)
    ap.add_argument("--folds", type=int, default=5)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32", "f64"])
    ap.add_argument("--dgp", default="tutorial", choices=["tutorial", "rct", "tutorial-rct"],
                    help="tutorial: the selection-biased df_mod at scale (default); rct: W "
                         "independent of X (the path solver's worst case)")
    ap.add_argument("--also-rct", type=int, default=1,
                    help="after the --dgp tutorial measurement, time the same step on the RCT "
                         "panel too (JSON key 'rct')")
    # weak (default): every GPU holds N=1e7 rows of the named config, so N=1 is exactly
    # the BASELINE config and rows/s measures the data-parallel design. The CV-LASSO
    # path solve is O(p^2 * lambdas) and independent of N, so at a fixed total N it is
    # an Amdahl term every rank repeats (use --scaling strong to measure that).
    ap.add_argument("--repeats", type=int, default=3,
                    help="> 1 (world 1): also time ate_dml(repeats=S) -- S distinct K-fold "
                         "partitions of K*K micro-segments from one Gram pass, median-aggregated "
                         "(JSON key 'repeated'; secondary, not the metric of record)")
    ap.add_argument("--scaling", default="weak", choices=["strong", "weak"])
    ap.add_argument("--seed", type=int, default=1991)
    ap.add_argument("--graph", type=int, default=-1,
                    help="capture the step in hipGraphs (default: on with a GPU; RCCL "
                         "collectives are captured inside them)")
    ap.add_argument("--parity", type=int, default=1,
                    help="after the timed steps, fit the same rows from a float64 panel (fp64 "
                         "Gram, fp64 path solves; untimed) and report the ATE / SE differences")
    ap.add_argument("--blocked", type=int, default=1,
                    help="1: 64-row blocked panel layout (one contiguous HBM run per Gram "
                         "K-step, ops/panel.py); 0: column-major")
    ap.add_argument("--exact", type=int, default=0,
                    help="1: world-size-invariant exact reduction mode (block-aligned row "
                         "shards, int64-limb Gram all-reduce, exact score moments: the same "
                         "ATE / SE bits at every world size; estimators/lasso.dml_phases)")
    ap.add_argument("--inflight", type=int, default=-1,
                    help="secondary throughput block: identical cross-fits in flight (one "
                         "hipGraph + stream + Gram workspace each); 1 = skip")
    return ap.parse_args()


def measure_inflight(args, comm, device, pan, inflight, fit_phases, agree, slot_comms_cache,
                     sync, single):
    """Secondary number: ``inflight`` independent cross-fits in flight (one hipGraph +
    stream + Gram workspace each, slots 1..inflight). The CV path solve is a latency-bound
    recurrence on few CUs, so another fit's HBM-bound Gram runs beside it. The fits are
    the same call on the same panel (identical bits, checked): this is the throughput of
    back-to-back calls, NOT the metric of record (that is the single call).
    Returns a dict for the JSON's "inflight" block."""
    import torch
    from ate_replication_causalml_amd.parallel import comm as C
    from ate_replication_causalml_amd.utils.graphs import Collective, SegmentedStep
    world = comm.world_size
    # One RCCL communicator per in-flight fit: collectives of ONE communicator must never
    # run concurrently (their kernels share its channel buffers, and graphs replayed on
    # different streams carry no order between them). Made once per process.
    if "slots" not in slot_comms_cache:
        slot_comms = [comm] * inflight
        if world > 1 and isinstance(comm, C.TorchComm) and comm.capturable:
            import torch.distributed as tdist
            slot_comms = [comm] + [C.TorchComm(tdist.new_group(list(range(world))))
                                   for _ in range(inflight - 1)]
            for c in slot_comms[1:]:
                c.barrier()             # create each communicator now, outside any capture
        slot_comms_cache["slots"] = slot_comms
    slot_comms = slot_comms_cache["slots"]
    # Gram workgroup count beside another fit's path solve (staggered: 824-4096 within 3 %,
    # profiles/r02_overlap/stagger_sweep.log; with the one-byte columns 1024: 2.98-2.99 ms per
    # fit, 2048: 3.02-3.04, 2560: 2.98-2.99, 3072: 3.01-3.03, profiles/r06_bench/inflight_wg)
    os.environ.setdefault("ATE_GRAM_PAIR_WG", "1024")
    # --stagger 2: the Grams of all fits run on one low-priority stream, each fit's remaining
    # phases on its own high-priority stream, so its path solve gets CUs ahead of the next
    # Gram's workgroups (eager stream hooks between the Gram graph and the rest)
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") \
        else (0, -1)
    gram_stream = torch.cuda.Stream(device, priority=lo)
    fit_streams = [torch.cuda.Stream(device, priority=hi) for _ in range(inflight)]
    fit_done = [None] * inflight

    def hooks(i):
        def to_gram(st):
            if fit_done[i] is not None:
                gram_stream.wait_event(fit_done[i])
            torch.cuda.set_stream(gram_stream)
            return st

        def to_fit(st):
            ev = torch.cuda.Event()
            ev.record(gram_stream)
            fit_streams[i].wait_event(ev)
            torch.cuda.set_stream(fit_streams[i])
            return st

        def done(st):
            ev = torch.cuda.Event()
            ev.record(fit_streams[i])
            fit_done[i] = ev
            return st
        return to_gram, to_fit, done

    def make_run(i):
        slot = i + 1
        phases = fit_phases(slot, slot_comms[i])
        to_gram, to_fit, done = hooks(i)
        # the one-kernel Gram phase as a plain launch, not a one-node graph: the fit's
        # reduce and the next Gram start ~55-65 us earlier (profiles/r05_eg)
        g0 = Collective(phases[0]) if os.environ.get("ATE_BENCH_EAGER_GRAM", "1") == "1" \
            else phases[0]
        phases = [Collective(to_gram), g0, Collective(to_fit), *phases[1:], Collective(done)]
        return SegmentedStep(phases, graph=True, agree=agree if world > 1 else None)

    home = torch.cuda.current_stream()
    runs = []
    try:
        for i in range(inflight):
            runs.append(make_run(i))
            torch.cuda.set_stream(home)     # stream-switching phases leave another current
        ok = agree(all(r.graphed for r in runs))
    except Exception as e:  # noqa: BLE001 - the secondary block is skipped, not fatal
        torch.cuda.set_stream(home)
        sync()
        print(f"[bench] in-flight block skipped: {e!r}", flush=True)
        ok = agree(False)
    finally:
        os.environ.pop("ATE_GRAM_PAIR_WG", None)
    if not ok:
        return None
    streams = [torch.cuda.Stream(device) for _ in runs]

    def run_step(k):
        i = k % len(runs)
        with torch.cuda.stream(streams[i]):
            return runs[i]()["res"]

    for k in range(max(args.warmup, len(runs))):
        run_step(k)
    sync()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    outs = []
    for k in range(args.steps):
        r = run_step(k)
        if k >= args.steps - len(runs):
            outs.append(r)
    sync()
    comm.barrier()
    sync()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
    comm.all_reduce_max_(el)
    ms = float(el.item()) / args.steps * 1e3
    outs = [o.detach().cpu() for o in outs]
    ref = single()["res"].detach().cpu()
    ate, se = (float(v) for v in outs[0])
    del runs
    return {"inflight": inflight, "ms_per_fit": ms, "rows_per_s": pan_rows(pan, comm) / (ms / 1e3),
            # the fits share one Gram plan (2048 workgroups: other row chunks than the single
            # call's plan, so other fp32 partial sums): equal to each other bit for bit, to the
            # single call up to the chunking's rounding
            "fits_agree": all(bool(torch.equal(o, outs[0])) for o in outs),
            "ate_hex": ate.hex(), "se_hex": se.hex(),
            "abs_diff_ate_vs_single": abs(ate - float(ref[0])),
            "rel_diff_se_vs_single": abs(se - float(ref[1])) / abs(float(ref[1])),
            "stagger": True,
            "communicators": len({id(c) for c in slot_comms}),
            "note": "throughput of identical back-to-back calls overlapped on streams; not "
                    "the metric of record"}


def pan_rows(pan, comm):
    import numpy as np
    from ate_replication_causalml_amd.estimators.lasso import global_seg_counts
    return float(np.asarray(global_seg_counts(pan, comm)).sum())


def measure(args, comm, device, dgp, n_total, slot_comms_cache):
    """Build the ``dgp`` panel, capture one ate_dml call, time ``args.steps`` calls back to
    back (the metric of record) and the median single-call latency, then the secondary
    in-flight throughput. Returns a dict (and the panel, for the parity refit)."""
    import torch
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.lasso import (EXACT_BLOCK, dml_phases,
                                                               global_seg_counts)
    from ate_replication_causalml_amd.ops.gram import plan_slot
    from ate_replication_causalml_amd.utils.graphs import Collective, SegmentedStep
    world, rank = comm.world_size, comm.rank

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize()

    sync()
    t_gen = time.perf_counter()
    pan = synthetic_panel(n_total, p=args.p, folds=args.folds, seed=args.seed, dtype=args.dtype,
                          blocked=bool(args.blocked) and args.dtype == "bf16",
                          device=device, rank=rank, world=world,
                          align=EXACT_BLOCK if args.exact else 0, dgp=dgp,
                          comm=comm if world > 1 else None)
    sync()
    t_gen = time.perf_counter() - t_gen
    seg_counts = global_seg_counts(pan, comm)   # fold sizes: data layout, fixed across steps
    use_graph = device.type == "cuda" if args.graph < 0 else bool(args.graph)
    exact = bool(args.exact)

    def agree(ok):
        t = torch.tensor([float(ok)], device=device)
        comm.all_reduce_min_(t)
        return bool(t.item())

    def in_slot(ph, i):
        if isinstance(ph, Collective):
            return ph

        def f(st):
            with plan_slot(i):  # eager calls too: never share another fit's workspace
                return ph(st)
        return f

    def fit_phases(slot, c):
        return [in_slot(ph, slot) for ph in dml_phases(
            pan, args.folds, "min", comm=c, seg_counts=seg_counts, exact=exact)]

    # ---- the metric of record: ONE ate_dml call as the library runs it --
    # its own captured step on one stream, the default Gram plan (whole rounds of
    # workgroups), slot 0's workspace. The K timed steps are K such calls back to back on
    # one stream (each call's Gram depends on nothing of the previous call's, but stream
    # order serialises them: no two fits overlap).
    saved = os.environ.pop("ATE_GRAM_PAIR_WG", None)
    try:
        with plan_slot(0):
            try:
                single = SegmentedStep(fit_phases(0, comm), graph=use_graph,
                                       agree=agree if world > 1 else None)
                err0 = None
            except Exception as e:  # noqa: BLE001 - reported, then every rank goes eager
                sync()
                single, err0 = None, repr(e)
    finally:
        if saved is not None:
            os.environ["ATE_GRAM_PAIR_WG"] = saved
    graphed = agree(single is not None and single.graphed) if use_graph else False
    if single is None or (use_graph and not graphed):
        # every rank falls back the same way
        print(f"[bench] rank {rank}: graph capture unavailable ({err0}); eager", flush=True)
        del single
        with plan_slot(0):
            single = SegmentedStep(fit_phases(0, comm), graph=False, warmup=0)
    graphs_per_fit = single.graph_count
    # world 1 has no collectives; at world > 1: whether every rank captured them
    collectives_captured = agree(single.collectives_captured) if world > 1 and graphed else None

    for k in range(args.warmup):
        res = single()["res"]
    sync()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(args.steps):
        res = single()["res"]
    sync()
    comm.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=device)
    comm.all_reduce_max_(el)
    elapsed = float(el.item())
    ate, se = [float(v) for v in res.detach().cpu()]
    if not (math.isfinite(ate) and math.isfinite(se)):
        from ate_replication_causalml_amd.utils.guards import NumericalError
        raise NumericalError(f"bench step returned ate={ate} se={se} (truncated CV fold path?)")
    ms = elapsed / args.steps * 1e3
    # latency of one call alone, each replay bracketed by device syncs (and a barrier):
    # median of >= 5 replays, the slowest rank per replay
    nlat = max(5, min(args.steps, 11))
    lats = []
    for k in range(nlat):
        sync()
        comm.barrier()
        t1 = time.perf_counter()
        single()
        sync()
        lats.append(time.perf_counter() - t1)
    lat_t = torch.tensor(lats, dtype=torch.float64, device=device)
    comm.all_reduce_max_(lat_t)
    lats = sorted(float(v) for v in lat_t.cpu())
    lat = lats[len(lats) // 2]

    inflight = 3 if args.inflight < 0 else max(1, args.inflight)
    inflight_out = None
    if inflight > 1 and device.type == "cuda" and graphed:
        inflight_out = measure_inflight(args, comm, device, pan, inflight, fit_phases, agree,
                                        slot_comms_cache, sync, single)
    out = {
        "dgp": dgp, "ms_per_step": ms, "rows_per_s": n_total / (ms / 1e3),
        "single_fit_ms": lat * 1e3, "single_fit_ms_all": [round(v * 1e3, 4) for v in lats],
        "single_fit_rows_per_s": n_total / lat,
        "ate": ate, "se": se, "ate_hex": ate.hex(), "se_hex": se.hex(),
        "n_kept": n_total, "n_generated": int(pan.n_generated) * 1,
        "panel_gen_s": t_gen, "hipgraph": graphed, "graphs_per_fit": graphs_per_fit,
        "collectives_captured": collectives_captured,
        "layout": ("blocked64" if pan.blocked else "colmajor") +
                  ("+bytes8" if getattr(pan, "bytes8", None) is not None else ""),
        "inflight": inflight_out,
    }
    if world > 1 and pan.selection is not None:
        out["n_generated"] = int(pan.selection.n_gen)
    del single
    return out, pan, seg_counts


def measure_repeated(args, comm, device, n_total, selection):
    """Repeated cross-fitting (estimators/lasso.dml_repeated_phases; Chernozhukov et al. 2018
    §3.4): the same kept rows in K*K micro-segments, ONE captured call = one Gram pass, S
    partitions' CV-LASSO paths and residual passes, the median aggregate. Timed like the
    main step (min(steps, 10) calls back to back after the warmup). Secondary: its
    fits_rows_per_s counts S fits per call, and the S split ATEs differ (distinct work)."""
    import torch
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.lasso import (dml_repeated_phases,
                                                               global_seg_counts)
    from ate_replication_causalml_amd.ops.gram import plan_slot
    from ate_replication_causalml_amd.utils.graphs import SegmentedStep
    K, S = args.folds, args.repeats
    pan = synthetic_panel(n_total, p=args.p, folds=K * K, seed=args.seed, dtype=args.dtype,
                          blocked=bool(args.blocked) and args.dtype == "bf16", device=device,
                          dgp=args.dgp, selection=selection)
    seg = global_seg_counts(pan, comm)
    use_graph = device.type == "cuda" if args.graph < 0 else bool(args.graph)
    with plan_slot(0):
        step = SegmentedStep(dml_repeated_phases(pan, K, S, "min", seg_counts=seg),
                             graph=use_graph)
    for _ in range(args.warmup):
        st = step()
    if device.type == "cuda":
        torch.cuda.synchronize()
    n = max(1, min(args.steps, 10))
    t0 = time.perf_counter()
    for _ in range(n):
        st = step()
    if device.type == "cuda":
        torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / n * 1e3
    ate, se = [float(v) for v in st["res"].detach().cpu()]
    splits = [[float(a), float(b)] for a, b in st["splits"].detach().cpu()]
    out = {"repeats": S, "folds": K, "micro_segments": K * K, "aggregate": "median",
           "ms_per_call": ms, "rows_per_s": n_total / (ms / 1e3),
           "fits_rows_per_s": S * n_total / (ms / 1e3), "ate": ate, "se": se,
           "splits": splits, "splits_distinct": len({a for a, _ in splits}) == S,
           "hipgraph": bool(step.graphed), "calls_timed": n}
    del step, pan
    return out


def main():
    args = parse()
    import torch
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from ate_replication_causalml_amd.parallel import comm as C
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.lasso import EXACT_BLOCK, dml_crossfit_panel
    from ate_replication_causalml_amd.ops.gram import clear_plans

    comm = C.from_env()
    emulate = int(os.environ.get("ATE_BENCH_EMULATE_WORLD", "0"))
    if emulate > 1 and comm.world_size == 1:
        # diagnostic only (tools/emulate_ranks.sh): rank 0's share of a world-W step on one
        # GPU -- its row shard, its path solves -- with no-op collectives (values are not
        # the world-W result; the JSON says "emulated_world")
        comm = C.EmulatedComm(0, emulate)   # plans the tutorial selection alone
    else:
        emulate = 0
    world, rank = comm.world_size, comm.rank
    if torch.cuda.is_available():
        torch.cuda.set_device(C.local_device())
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    n_total = int(args.rows) * (world if args.scaling == "weak" else 1)

    from ate_replication_causalml_amd.utils.guards import collective_timeout
    # a dead peer must end the job with a message, not hang the other ranks in RCCL
    guard = collective_timeout(float(os.environ.get("ATE_COLLECTIVE_TIMEOUT", "900")),
                               "bench step") if world > 1 else contextlib.nullcontext()
    guard.__enter__()
    cache = {}
    main_m, pan, seg_counts = measure(args, comm, device, args.dgp, n_total, cache)
    parity = None
    if args.parity and args.dtype != "f64":
        # ATE/SE parity (the metric's second half), untimed: the same kept rows generated as
        # a float64 panel (the selection plan is reused: same rows), fp64 Gram and fp64 path
        # solves (the path tests/test_gpu.py pins against the float64 reference estimator)
        clear_plans()
        t2 = time.perf_counter()
        pan64 = synthetic_panel(n_total, p=args.p, folds=args.folds, seed=args.seed,
                                dtype="f64", device=device, rank=rank, world=world,
                                align=EXACT_BLOCK if args.exact else 0,
                                dgp=args.dgp, selection=pan.selection)
        r64 = dml_crossfit_panel(pan64, args.folds, "min", comm=comm, seg_counts=seg_counts)[0]
        a64, s64 = [float(v) for v in r64.detach().cpu()]
        ate, se = main_m["ate"], main_m["se"]
        parity = {"reference": "same kept rows as a float64 panel: fp64 Gram + fp64 CV-LASSO "
                               "paths", "dgp": args.dgp,
                  "ate_f64": a64, "se_f64": s64, "abs_diff_ate": abs(ate - a64),
                  "abs_diff_ate_in_se": abs(ate - a64) / abs(s64),
                  "rel_diff_se": abs(se - s64) / abs(s64),
                  "within_tolerance": bool(abs(ate - a64) <= 0.01 * abs(s64)
                                           and abs(se - s64) <= 1e-3 * abs(s64)),
                  "tolerance": "|dATE| <= 0.01 SE_f64 and |dSE| <= 1e-3 SE_f64",
                  "seconds": time.perf_counter() - t2}
        del pan64
        clear_plans()
    repeated = None
    if args.repeats > 1 and world == 1 and not emulate:
        clear_plans()
        repeated = measure_repeated(args, comm, device, n_total, pan.selection)
        clear_plans()
    del pan
    rct = None
    if args.also_rct and args.dgp != "rct":
        clear_plans()
        if device.type == "cuda":
            torch.cuda.empty_cache()
        rct, rpan, _ = measure(args, comm, device, "rct", n_total, cache)
        del rpan
        clear_plans()
    guard.__exit__(None, None, None)
    ms = main_m["ms_per_step"]
    rows_per_s = n_total / (ms / 1e3)
    if rank == 0:
        out = {
            "metric": "rows/sec for DML-ATE cross-fit, N=1e7 p=500, 1/2/4/8 MI355X; ATE/SE parity",
            "value": rows_per_s,
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": rows_per_s / CPU_BASELINE_ROWS_PER_S,
            "baseline": "CPU bound: fp32 fold Grams alone, 8-core host (BASELINE.md)",
            "dtype": args.dtype,
            "data": ("synthetic: the tutorial's selection-biased df_mod at scale (calibrated "
                     "latent-voter DGP + ate_replication.Rmd:97-121 transform over generated "
                     "rows), generated on device" if args.dgp == "tutorial" else
                     f"synthetic ({args.dgp} panel, tutorial DGP shape, generated on device)"),
            "config": {
                "model": "DML-PLR 5-fold cross-fit, CV-LASSO nuisances (100 lambdas, inner 4-fold CV)",
                "global_batch": n_total,
                "seq_len": args.p,
                "N": n_total,
                "p": args.p,
                "folds": args.folds,
                "parallelism": f"dp{world}",
                "dgp": args.dgp,
                "n_kept": n_total,
                "n_generated": main_m["n_generated"],
                "layout": main_m["layout"],
                "timed_step": "one ate_dml call (SURVEY.md 7.5), calls back to back on one "
                              "stream, no two fits overlapping",
            },
            "ate": main_m["ate"],
            "se": main_m["se"],
            "ate_hex": main_m["ate_hex"],
            "se_hex": main_m["se_hex"],
            "hipgraph": main_m["hipgraph"],
            "single_fit_ms": main_m["single_fit_ms"],
            "single_fit_ms_all": main_m["single_fit_ms_all"],
            "single_fit_rows_per_s": main_m["single_fit_rows_per_s"],
            "graphs_per_fit": main_m["graphs_per_fit"],
            "exact": bool(args.exact),
            "collectives_captured": main_m["collectives_captured"],
            "panel_gen_s": main_m["panel_gen_s"],
            "throughput_inflight": main_m["inflight"],
            "parity": parity,
            "repeated": repeated,
            "rct": None if rct is None else {k: rct[k] for k in (
                "ms_per_step", "rows_per_s", "single_fit_ms", "single_fit_ms_all",
                "single_fit_rows_per_s", "ate", "se", "ate_hex", "se_hex", "hipgraph",
                "inflight")},
        }
        if emulate > 1:
            out["emulated_world"] = emulate
        print(json.dumps(out), flush=True)
    if world > 1 and not emulate:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
