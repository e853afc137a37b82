"""Shared plumbing for the device estimators: input coercion, device choice,
result read-back (one host sync per estimator)."""
from __future__ import annotations

import numpy as np
import torch

from ..result import AteResult


def default_device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device("cpu")


def resolve_device(device=None) -> torch.device:
    if device is None:
        return default_device()
    return torch.device(device)


def as_np(a) -> np.ndarray:
    if isinstance(a, torch.Tensor):
        return a.detach().double().cpu().numpy()
    return np.asarray(a, dtype=np.float64)


def read_result(res: torch.Tensor, method: str, **diag) -> AteResult:
    v = res.detach().double().cpu().numpy()
    return AteResult.make(method, v[0], v[1] if len(v) > 1 else None, **diag)
