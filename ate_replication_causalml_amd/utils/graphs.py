"""hipGraph capture of device-only estimator steps ("every ate_*() is
one hipGraph launch").

``GraphedStep(fn)`` runs ``fn`` eagerly ``warmup`` times (so plans, workspaces and the
device-constant cache are populated: no allocation or host->device copy is left in
the steady state), captures one call with ``torch.cuda.graph`` on a side stream, and
replays it: the whole cross-fit — Gram launches, the CV path launch with its
device-side progress flags, selection, residual pass, moments, finalisation — is one
graph launch. Iterative solvers in the step use fixed launch budgets with device
convergence flags (ops/linalg.logistic_irls), so nothing in them needs the host.
``fn`` must return tensors; they are the graph's static outputs (overwritten on
every replay).

A graph holds raw device addresses of every workspace it touched. Caches that can
evict (Gram plans, device constants) call :func:`pin` for each object they hand out;
during a capture the object is appended to the capturing step's pin list, so an
eviction only drops the cache's reference and the memory lives as long as the graph.

``SegmentedStep`` is the multi-GPU form: a list of phases, each either a device-only
callable or a :class:`Collective`. RCCL collectives (``capturable=True``: enqueued on
the current HIP stream by torch's ``nccl`` backend) are captured INTO the graph with the
device phases around them, so a world-W cross-fit is one graph launch like a world-1
one. Host-side phases (gloo collectives, stream-switch hooks) are
never captured: they run eagerly between the graphs of the device runs around them.
If capturing the collectives fails, the step falls back to graphs of the device runs
with every collective eager between them, and prints why.
"""
from __future__ import annotations

import contextlib
import gc

import torch

_pins: list | None = None


@contextlib.contextmanager
def _no_gc():
    """Python's cyclic GC must not run inside a stream capture: an evicted graph reclaimed
    there destroys its executable / frees its pool while the stream is capturing, which
    HIP rejects (an error raised in a destructor aborts the process)."""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def pin(obj):
    """Keep ``obj`` alive for the lifetime of the graph being captured (no-op otherwise)."""
    if _pins is not None:
        _pins.append(obj)
    return obj


class GraphedStep:
    def __init__(self, fn, warmup: int = 1):
        global _pins
        self.fn = fn
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        prev, _pins = _pins, []
        try:
            gc.collect()            # reclaim evicted graphs here, outside the capture
            with _no_gc(), torch.cuda.graph(self.graph):
                self.out = fn()
            self.pins = _pins
        finally:
            _pins = prev
        torch.cuda.synchronize()

    def __call__(self):
        self.graph.replay()
        return self.out


def maybe_graphed(fn, enable: bool, warmup: int = 1):
    """GraphedStep when enabled and capture succeeds, else the eager function."""
    if not enable or not torch.cuda.is_available():
        return fn, False
    try:
        return GraphedStep(fn, warmup), True
    except Exception as e:  # noqa: BLE001 - fall back to eager, but say why
        print(f"[graphs] capture failed, running eagerly: {e}", flush=True)
        torch.cuda.synchronize()
        return fn, False


class Collective:
    """A phase of a :class:`SegmentedStep` that talks to other ranks (or switches streams).
    ``capturable``: it only enqueues work on the current HIP stream (an RCCL all-reduce),
    so it may be captured inside the graph of the device phases around it; otherwise it
    runs eagerly between graph replays."""

    def __init__(self, fn, capturable: bool = False):
        self.fn = fn
        self.capturable = capturable

    def __call__(self, state):
        return self.fn(state)


def _fuse(phases, fuse_collectives=False):
    """Merge runs of consecutive device phases into one phase (one graph per run: with
    no collectives in between, e.g. world size 1, the whole step is a single graph).
    ``fuse_collectives``: capturable collectives join the runs."""
    out, run = [], []

    def flush():
        if run:
            fns = tuple(run)

            def composed(st, fns=fns):
                for f in fns:
                    st = f(st)
                return st
            out.append(composed)
            run.clear()

    for ph in phases:
        if isinstance(ph, Collective) and not (fuse_collectives and ph.capturable):
            flush()
            out.append(ph)
        else:
            run.append(ph)
    flush()
    return out


class SegmentedStep:
    """A step split into phases ``fn(state) -> state``. Device phases (and capturable
    collectives, when ``capture_collectives``) are captured in one graph per run between
    host-side phases; host-side :class:`Collective` phases run eagerly on the current
    stream between replays. ``state`` is whatever the phases pass along (tensors whose
    storage is static across calls: graph outputs are overwritten in place on replay).

    Capture runs the phases ``warmup`` times eagerly first (populating plans, constants
    and RCCL communicators), then captures each run given the state produced by the
    phases before it. If a run with collectives in it cannot be captured, the step is
    rebuilt with every collective eager (reason printed, ``fallback_reason``). The
    step's result is the last phase's state. ``graph_count``: graphs replayed per call;
    ``collectives_captured``: whether collectives sit inside the graphs."""

    def __init__(self, phases, graph: bool, warmup: int = 1, capture_collectives: bool = True,
                 agree=None):
        """``agree(ok: bool) -> bool`` (multi-rank steps): the minimum of ``ok`` over the
        ranks. The graphs holding collectives are captured WITHOUT replaying them, every
        rank reports whether its capture succeeded, and only when all did are they replayed;
        otherwise every rank rebuilds with eager collectives. No collective of the attempt
        has then run anywhere, so the ranks' collective sequences stay paired."""
        self.raw = list(phases)
        self.fallback_reason = None
        has_cc = any(isinstance(p, Collective) and p.capturable for p in self.raw)
        self.phases = _fuse(self.raw)
        self.graphs = [None] * len(self.phases)
        self.pins = []
        self.collectives_captured = False
        for _ in range(warmup):
            self._eager()
        if not graph:
            return
        if capture_collectives and has_cc:
            ok, err = True, None
            try:
                self._capture(_fuse(self.raw, fuse_collectives=True), replay=False)
            except Exception as e:  # noqa: BLE001 - fall back, but say why
                ok, err = False, e
            if agree is not None:
                ok = bool(agree(ok))
                if err is None and not ok:
                    err = RuntimeError("another rank could not capture its collectives")
            if ok:
                self()                  # first execution: every rank, same collectives
                torch.cuda.synchronize()
                self.collectives_captured = True
                return
            self.fallback_reason = repr(err)
            print(f"[graphs] capturing the collectives failed, they run eagerly between "
                  f"graph segments: {err}", flush=True)
            torch.cuda.synchronize()
            self.phases = _fuse(self.raw)
            self.graphs = [None] * len(self.phases)
            self.pins = []
        self._capture(_fuse(self.raw))

    def _capture(self, phases, replay: bool = True):
        """Capture every device run of ``phases``. ``replay``: replay each graph right
        after its capture (capture does not execute) so later eager phases see its
        outputs; without it, the graphs are only recorded (their outputs' storage is all
        that later captures need) and the first call executes them."""
        global _pins
        torch.cuda.synchronize()
        graphs = [None] * len(phases)
        pins = []
        state = None
        for i, ph in enumerate(phases):
            if isinstance(ph, Collective):
                state = ph(state)
                continue
            g = torch.cuda.CUDAGraph()
            prev, _pins = _pins, []
            try:
                gc.collect()
                with _no_gc(), torch.cuda.graph(g):
                    out = ph(state)
                pins += _pins
            finally:
                _pins = prev
            graphs[i] = (g, out)
            torch.cuda.synchronize()
            if replay:
                g.replay()      # capture does not execute: produce the state for later phases
            state = out
        torch.cuda.synchronize()
        self.phases, self.graphs, self.pins = phases, graphs, pins

    @property
    def graphed(self) -> bool:
        return any(g is not None for g in self.graphs)

    @property
    def graph_count(self) -> int:
        return sum(g is not None for g in self.graphs)

    def _eager(self):
        state = None
        for ph in self.phases:
            state = ph(state)
        return state

    def __call__(self):
        state = None
        for ph, g in zip(self.phases, self.graphs):
            if g is None:
                state = ph(state)
            else:
                g[0].replay()
                state = g[1]
        return state


def _data(x):
    """The device buffer behind an estimator input (a tensor, or a DevicePanel's data)."""
    return x if isinstance(x, torch.Tensor) else x.data


def layout_key(*inputs):
    """Everything a captured body's launch sequence depends on: tensor shapes / dtypes /
    devices and, for panels, the column map, fold segments and real-row counts."""
    key = []
    for x in inputs:
        if x is None:                 # optional input (e.g. no exact-split value table)
            key.append(None)
            continue
        t = _data(x)
        k = (tuple(t.shape), t.dtype, str(t.device))
        if not isinstance(x, torch.Tensor):
            k += (x.n, tuple(sorted(x.cols.items())), tuple(map(tuple, x.seg_bounds)),
                  tuple(int(c) for c in x.seg_nreal), bool(getattr(x, "identity", False)),
                  getattr(x, "bytes8", None) is not None)
        key.append(k)
    return tuple(key)


class _Captured:
    """``body(*inputs)`` captured once over STATIC inputs (an earlier call's own tensors /
    panels, kept alive here); a later call copies its data into them and replays."""

    def __init__(self, body, inputs, static_args, warmup):
        self.inputs = inputs = list(inputs)
        # the closure holds the input list, not self: no reference cycle, so an evicted
        # entry (and its graph) is freed at once, outside any capture
        self.step = GraphedStep(lambda: body(*inputs, *static_args), warmup)

    def load(self, inputs):
        for s, x in zip(self.inputs, inputs):
            if x is not s and x is not None:
                _data(s).copy_(_data(x))
                if getattr(x, "bytes8", None) is not None:      # a panel's one-byte columns
                    s.bytes8.copy_(x.bytes8)

    def __call__(self, inputs):
        self.load(inputs)
        return self.step()


class _Seen:
    """First call of a key: it ran eagerly on these inputs. Small inputs are kept and
    become the graph's static inputs on the second call (``inputs``); inputs above the
    cache's retention threshold are not kept (``inputs is None``): the second call's own
    buffers are captured instead, so a one-off call on a large panel holds no HBM."""

    def __init__(self, inputs):
        self.inputs = None if inputs is None else list(inputs)


def _nbytes(inputs):
    tot = 0
    for x in inputs:
        if x is None:
            continue
        t = _data(x)
        tot += t.numel() * t.element_size()
    return tot


def _env_bytes(name, default):
    import os
    v = os.environ.get(name)
    return int(float(v)) if v else default


class GraphCache:
    """Per-estimator hipGraph cache (SURVEY.md §7.1 "every ate_*() is one hipGraph
    launch"). ``run(name, body, inputs, *static_args)`` calls ``body(*inputs,
    *static_args)`` -- a device-only function of the inputs (fixed launch budgets, device
    flags, cached constants; no host sync). Per (name, static args, input layout):

    * 1st call: runs eagerly; its input buffers are kept when they are small
      (``retain_bytes``), so a one-off call on a large panel keeps nothing;
    * 2nd call: copies its data into the kept buffers (or keeps its own), runs the body
      once eagerly on them (re-populating plan / constant caches that may have been
      evicted in between), captures it and replays it;
    * later calls: copy + ONE graph launch.

    LRU bounded by ``maxsize`` entries (32: the 14-row tutorial pass alone keeps more than
    8 estimator layouts, and an LRU of 8 recaptured several of them on every pass) and
    ``max_bytes`` of retained input buffers
    (``ATE_GRAPH_CACHE_BYTES``, default 24 GiB; each entry also holds its graph's memory
    pool). A body that cannot be captured is remembered and runs eagerly from then on
    (the reason is printed). Outputs of a replay are the graph's static tensors: read them
    before the next call. ``clear()`` drops every entry (and its HBM).
    Returns (output, replayed: bool)."""

    def __init__(self, maxsize: int = 32, max_bytes: int | None = None,
                 retain_bytes: int | None = None):
        self.maxsize = maxsize
        self.max_bytes = max_bytes if max_bytes is not None else \
            _env_bytes("ATE_GRAPH_CACHE_BYTES", 24 << 30)
        self.retain_bytes = retain_bytes if retain_bytes is not None else \
            _env_bytes("ATE_GRAPH_RETAIN_BYTES", 1 << 30)
        self.entries: dict = {}
        self.sizes: dict = {}
        self.eager: set = set()

    @property
    def held_bytes(self):
        return sum(self.sizes.values())

    def _evict(self, need=0):
        while self.entries and (len(self.entries) >= self.maxsize or
                                self.held_bytes + need > self.max_bytes):
            k = next(iter(self.entries))
            self.entries.pop(k)
            self.sizes.pop(k, None)

    def run(self, name, body, inputs, *static_args):
        key = (name, static_args, layout_key(*inputs))
        if key in self.eager:
            return body(*inputs, *static_args), False
        g = self.entries.pop(key, None)
        self.sizes.pop(key, None)
        nb = _nbytes(inputs)
        if g is None:
            keep = nb <= self.retain_bytes and nb <= self.max_bytes
            self._evict(nb if keep else 0)
            self.entries[key] = _Seen(inputs if keep else None)
            self.sizes[key] = nb if keep else 0
            return body(*inputs, *static_args), False
        if isinstance(g, _Seen):
            if nb > self.max_bytes:
                # too large to hold for a replay: run eagerly, stay "seen"
                self.entries[key] = g
                self.sizes[key] = 0
                return body(*inputs, *static_args), False
            self._evict(nb)
            static = g.inputs if g.inputs is not None else list(inputs)
            try:
                torch.cuda.synchronize()
                for s, x in zip(static, inputs):
                    if x is not s and x is not None:
                        _data(s).copy_(_data(x))
                        if getattr(x, "bytes8", None) is not None:
                            s.bytes8.copy_(x.bytes8)
                g = _Captured(body, static, static_args, warmup=1)
            except Exception as e:  # noqa: BLE001 - fall back to eager, but say why
                print(f"[graphs] {name}: capture failed, running eagerly: {e}", flush=True)
                torch.cuda.synchronize()
                self.eager.add(key)
                return body(*inputs, *static_args), False
        self.entries[key] = g
        self.sizes[key] = nb
        return g(inputs), True

    def drop(self, name, inputs, *static_args):
        """Forget the entry of (name, static args, input layout): its next call starts over."""
        key = (name, static_args, layout_key(*inputs))
        self.entries.pop(key, None)
        self.sizes.pop(key, None)
        self.eager.discard(key)

    def clear(self):
        self.entries.clear()
        self.sizes.clear()
        self.eager.clear()


estimator_graphs = GraphCache()


def clear_graph_caches():
    """Release every cached graph, its retained input buffers and the Gram plans (HBM held
    between estimator calls); call between phases of a long job or at teardown."""
    estimator_graphs.clear()
    try:
        from ..ops.gram import clear_plans
        clear_plans()
    except Exception:  # noqa: BLE001 - nothing to clear without the ops module
        pass
    if torch.cuda.is_available():
        torch.cuda.empty_cache()
