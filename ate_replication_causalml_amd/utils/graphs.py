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
"""
from __future__ import annotations

import torch


class GraphedStep:
    def __init__(self, fn, warmup: int = 1):
        self.fn = fn
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = fn()
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
