"""Synthetic data with the tutorial's schema.

The reference reads the Gerber-Green-Larimer social-pressure CSV
(``ate_replication.Rmd:32-34``), which is not shipped (``.gitignore:6``).
This module generates data with the same schema: 15 continuous covariates
(standardised with ``scale()``, ``ate_replication.Rmd:72-74``), 6 binary
covariates, binary outcome ``Y`` (``outcome_voted``) and binary treatment ``W``
(``treat_neighbors``), in the reference column order (cts, bin, Y, W;
``ate_replication.Rmd:90-93``).

Every draw is a Philox function of (seed, column stream, row index), so the
same rows can be produced on the host (this file) or directly in HBM by the
``dgp_fill`` HIP kernel for the scaled configs (N up to 1e8, p up to 2000),
without ever materialising the panel on the host.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ..parallel import rng

CTS_NAMES = [
    "yob", "city", "hh_size", "totalpopulation_estimate", "percent_male", "median_age",
    "percent_62yearsandover", "percent_white", "percent_black", "percent_asian",
    "median_income", "employ_20to64", "highschool", "bach_orhigher",
    "percent_hispanicorlatino",
]  # ate_replication.Rmd:49-55
BIN_NAMES = ["sex", "g2000", "g2002", "p2000", "p2002", "p2004"]  # ate_replication.Rmd:56
COVARIATES = CTS_NAMES + BIN_NAMES  # ate_replication.Rmd:57

# DGP constants (calibrated so that n=50,000 gives roughly the published
# oracle ~0.096, naive ~0.003 and ~41k dropped rows).
S_CTS = 0           # streams 0..14: continuous covariates
S_FACTOR = 40       # shared census-block factor for the neighbourhood covariates
S_LATENT = 41       # latent propensity to vote
S_HIST = 50         # 50..54 vote history g2000..p2004
S_SEX = 60
S_W = 61
S_Y = 62
S_EXTRA = 100       # 100.. extra nuisance columns for scaled configs

INTERCEPT = -1.4
B_HIST = 0.3
B_LATENT = 0.2
TAU_LOGIT = 0.45
P_TREAT = 1.0 / 6.0
HIST_THRESH = 0.6
HIST_LATENT = 0.5
YOB_LATENT = 0.3
FACTOR_LOAD = 0.6


def _normal(seed, stream, idx):
    return rng.normal_pair(seed, rng.P_DGP, stream, idx)[0]


def _uniform(seed, stream, idx):
    return rng.uniform(seed, rng.P_DGP, stream, idx)


@dataclass
class TutorialData:
    X: np.ndarray          # (n, p) float64, columns named by ``names``
    W: np.ndarray          # (n,) float64 in {0,1}
    Y: np.ndarray          # (n,) float64 in {0,1}
    names: list
    tau_true: float        # population ATE on the probability scale (MC of the DGP)

    @property
    def n(self):
        return self.X.shape[0]

    def to_frame(self):
        import pandas as pd
        df = pd.DataFrame(self.X, columns=self.names)
        df["Y"] = self.Y
        df["W"] = self.W
        return df


def raw_columns(n: int, seed: int, p_extra: int = 0, row_offset: int = 0):
    """Unscaled draws for rows [row_offset, row_offset+n)."""
    idx = np.arange(row_offset, row_offset + n, dtype=np.uint64)
    f = _normal(seed, S_FACTOR, idx)
    cts = np.empty((n, 15))
    for j in range(15):
        z = _normal(seed, S_CTS + j, idx)
        cts[:, j] = z if j < 3 else FACTOR_LOAD * f + np.sqrt(1 - FACTOR_LOAD ** 2) * z
    latent = _normal(seed, S_LATENT, idx) + YOB_LATENT * cts[:, 0]
    hist = np.empty((n, 5))
    for k in range(5):
        hist[:, k] = (_normal(seed, S_HIST + k, idx) + HIST_LATENT * latent > HIST_THRESH)
    sex = (_uniform(seed, S_SEX, idx) < 0.5).astype(np.float64)
    W = (_uniform(seed, S_W, idx) < P_TREAT).astype(np.float64)
    eta = INTERCEPT + B_HIST * hist.sum(1) + B_LATENT * latent
    Y = (_uniform(seed, S_Y, idx) < 1.0 / (1.0 + np.exp(-(eta + TAU_LOGIT * W)))).astype(np.float64)
    tau_i = 1 / (1 + np.exp(-(eta + TAU_LOGIT))) - 1 / (1 + np.exp(-eta))
    extra = np.empty((n, p_extra))
    for j in range(p_extra):
        z = _normal(seed, S_EXTRA + j, idx)
        if j % 4 == 3:   # every 4th extra column is binary
            extra[:, j] = (z > 0).astype(np.float64)
        else:
            extra[:, j] = FACTOR_LOAD * f + np.sqrt(1 - FACTOR_LOAD ** 2) * z
    return cts, np.column_stack([sex, hist]), extra, W, Y, tau_i


def r_scale(a: np.ndarray) -> np.ndarray:
    """R ``scale()``: centre and divide by the sample SD (n-1 denominator)."""
    m = a.mean(0)
    s = a.std(0, ddof=1)
    s = np.where(s > 0, s, 1.0)
    return (a - m) / s


def make_tutorial_data(n: int = 50_000, seed: int = 1991, p_extra: int = 0) -> TutorialData:
    """The ``df`` of ``ate_replication.Rmd:89-94`` (scaled cts + binary + Y + W)."""
    cts, binc, extra, W, Y, tau_i = raw_columns(n, seed, p_extra)
    cts = r_scale(cts)
    names = list(COVARIATES)
    blocks = [cts, binc]
    if p_extra:
        ex = extra.copy()
        cont = [j for j in range(p_extra) if j % 4 != 3]
        ex[:, cont] = r_scale(ex[:, cont])
        blocks.append(ex)
        names += [f"x_extra{j}" for j in range(p_extra)]
    X = np.column_stack(blocks)
    return TutorialData(X=X, W=W, Y=Y, names=names, tau_true=float(tau_i.mean()))
