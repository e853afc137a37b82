"""Device-resident constants keyed by content.

Small host-built index/mask/parameter arrays (column lists, fold masks, problem
descriptors) are uploaded once per (device, dtype, content) and reused, so a
steady-state estimator call performs no host->device copies — a prerequisite for
capturing it in a hipGraph (utils/graphs.py) and a saving of one synchronous
pageable copy per array per call otherwise.
"""
from __future__ import annotations

import hashlib

import numpy as np
import torch

from ..utils.graphs import pin

_CACHE: dict = {}
_MAX = 4096


def const(values, dtype, device) -> torch.Tensor:
    a = np.ascontiguousarray(np.asarray(values))
    dev = torch.device(device)
    if dev.type != "cuda":
        return torch.as_tensor(a.copy()).to(dtype)
    key = (str(dev), str(dtype), a.dtype.str, a.shape, hashlib.sha1(a.tobytes()).hexdigest())
    t = _CACHE.get(key)
    if t is None:
        if len(_CACHE) >= _MAX:
            _CACHE.clear()
        t = torch.as_tensor(a).to(device=dev, dtype=dtype)
        _CACHE[key] = t
    # a graph capturing this constant keeps it alive even if the cache is cleared later
    return pin(t)


def const_bytes(raw: np.ndarray, device) -> torch.Tensor:
    """Structured / raw-byte arrays (e.g. EnetProblem records) as a uint8 tensor."""
    return const(np.ascontiguousarray(raw).view(np.uint8).reshape(-1), torch.uint8, device)
