"""Failure detection.

The reference's only defences are ``na.omit`` (ate_replication.Rmd:93), propensity
clipping (ate_functions.R:181-182) and ``mean(..., na.rm=TRUE)``
(ate_functions.R:186,243,281). Here:

* ``check_finite`` raises a NumericalError naming the tensor (device-side count,
  one scalar read);
* ``overlap_report`` counts propensities at/near 0 or 1 and the effective sample
  size of the inverse-propensity weights — returned with the estimate so a user sees
  a positivity problem instead of a silently huge SE;
* ``collective_timeout`` arms a watchdog around a distributed phase: if a peer rank
  dies, the surviving ranks abort with a clear message instead of hanging in RCCL.
"""
from __future__ import annotations

import contextlib
import os
import threading

import torch


class NumericalError(RuntimeError):
    pass


def check_finite(name: str, t: torch.Tensor):
    bad = int((~torch.isfinite(t)).sum())
    if bad:
        raise NumericalError(f"{name}: {bad} non-finite value(s) of {t.numel()}")
    return t


def overlap_report(p: torch.Tensor, w: torch.Tensor | None = None, eps: float = 1e-3) -> dict:
    p = p.double()
    ipw = 1.0 / torch.where(w > 0.5, p, 1 - p) if w is not None else 1.0 / (p * (1 - p))
    ess = float(ipw.sum() ** 2 / (ipw ** 2).sum())
    return {"p_min": float(p.min()), "p_max": float(p.max()),
            "n_p_extreme": int(((p < eps) | (p > 1 - eps)).sum()),
            "n_p_exact01": int(((p == 0) | (p == 1)).sum()), "ipw_ess": ess}


@contextlib.contextmanager
def collective_timeout(seconds: float | None = None, what: str = "collective"):
    """Abort the process (exit code 3) if the body does not finish in time."""
    seconds = seconds or float(os.environ.get("ATE_COLLECTIVE_TIMEOUT", "600"))
    done = threading.Event()

    def watchdog():
        if not done.wait(seconds):
            rank = os.environ.get("RANK", "?")
            print(f"[rank {rank}] {what} did not complete in {seconds:.0f}s; a peer likely "
                  f"failed — aborting", flush=True)
            os._exit(3)

    th = threading.Thread(target=watchdog, daemon=True)
    th.start()
    try:
        yield
    finally:
        done.set()
