"""Loader for the reference's real input (ate_replication.Rmd:33-94): the
social-pressure GOTV file ``socialpresswgeooneperhh_NEIGH.csv``.

Not shipped (no network here); users who have it get the same ``df`` the driver
builds: ``sample_n(n_obs)`` -> select covariates + outcome_voted + treat_neighbors ->
``scale()`` the 15 continuous columns -> rename to Y/W -> ``na.omit``. The row sample is
R's own draw by default (``sampler="r"``: ``set.seed(seed); sample_n(df, n_obs)`` with R's
Mersenne-Twister and rejection sampler, parallel/rrng.py), in R's sampled row order -- the
order the selection transform's "first 85%" rule (Q18) sees. ``sampler="philox"`` uses a
counter-based Philox permutation (purpose P_SAMPLE_ROWS) kept in file order instead.
"""
from __future__ import annotations

import numpy as np
import torch

from ..parallel import rng
from .dgp import BIN_NAMES, CTS_NAMES, TutorialData, r_scale

OUTCOME, TREATMENT = "outcome_voted", "treat_neighbors"


def load_social_pressure(path, n_obs: int = 50_000, seed: int = 1991,
                         device=None, sampler: str = "r") -> TutorialData:
    """``device="cuda"`` standardises on the GPU (K02, csrc/prep.hip); same formulas."""
    import pandas as pd
    cols = list(CTS_NAMES) + list(BIN_NAMES) + [OUTCOME, TREATMENT]
    raw = pd.read_csv(path, usecols=cols)
    n = len(raw)
    if sampler == "r":
        from ..parallel.rrng import r_sample_rows
        raw = raw.iloc[r_sample_rows(n, min(n_obs, n), seed)]
    elif n_obs < n:
        r = rng.random_u32(seed, rng.P_SAMPLE_ROWS, 0, np.arange(n, dtype=np.uint64))
        keys = (r[:, 0].astype(np.uint64) << np.uint64(32)) | r[:, 1].astype(np.uint64)
        take = np.sort(np.argsort(keys, kind="stable")[:n_obs])
        raw = raw.iloc[take]
    sub = raw[cols].astype(np.float64)
    cts = sub[list(CTS_NAMES)].to_numpy()
    # R scale() ignores NA within a column; rows with any NA are dropped afterwards
    if device is not None and torch.device(device).type == "cuda":
        from ..ops.prep import r_scale as dev_scale
        cts = dev_scale(torch.as_tensor(cts, device=device), constant_to_one=True).cpu().numpy()
    else:
        cm = np.nanmean(cts, 0)
        cs = np.nanstd(cts, 0, ddof=1)
        cts = (cts - cm) / np.where(cs > 0, cs, 1.0)
    X = np.column_stack([cts, sub[list(BIN_NAMES)].to_numpy()])
    Y = sub[OUTCOME].to_numpy()
    W = sub[TREATMENT].to_numpy()
    ok = np.isfinite(X).all(1) & np.isfinite(Y) & np.isfinite(W)
    return TutorialData(X=X[ok], W=W[ok], Y=Y[ok], names=list(CTS_NAMES) + list(BIN_NAMES),
                        tau_true=float("nan"))


__all__ = ["load_social_pressure", "r_scale"]
