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

S_CTS = 0           # streams 0..14: continuous covariates
S_FACTOR = 40       # shared census-block factor for the neighbourhood covariates
S_LATENT = 41       # latent propensity to vote
S_HIST = 50         # 50..54 vote history g2000..p2004
S_SEX = 60
S_W = 61
S_Y = 62
S_EXTRA = 100       # 100.. extra nuisance columns for scaled configs


@dataclass(frozen=True)
class DgpParams:
    """Constants of the latent-voter model: 15 N(0,1) continuous
    covariates (3 individual, 12 loading on a census-block factor), latent = N(0,1) +
    yob_latent * yob, vote history k = 1[N(0,1) + hist_latent * latent > hist_thresh[k]]
    (g2000, g2002, p2000, p2002, p2004), sex ~ Bern(0.5), W ~ Bern(p_treat) (the RCT),
    Y ~ Bern(sigmoid(intercept + b_hist' history + b_latent * latent + tau_logit * W))."""
    intercept: float = -1.4
    b_hist: tuple = (0.3, 0.3, 0.3, 0.3, 0.3)
    b_latent: float = 0.2
    tau_logit: float = 0.45
    p_treat: float = 1.0 / 6.0
    hist_thresh: tuple = (0.6, 0.6, 0.6, 0.6, 0.6)
    hist_latent: float = 0.5
    yob_latent: float = 0.3
    factor_load: float = 0.6

    def device_block(self) -> np.ndarray:
        """The float64[18] parameter block of csrc/dgp.hip (load_params: the selection
        rule's parameters used at full precision, the rest rounded to fp32 there)."""
        fl = self.factor_load
        return np.array([self.intercept, *self.b_hist, self.b_latent, self.tau_logit,
                         self.p_treat, *self.hist_thresh, self.hist_latent, self.yob_latent,
                         fl, np.sqrt(1 - fl ** 2)], dtype=np.float64)


# The scaled-config panels (data/device_dgp.synthetic_panel, the bench) and the HIP
# generator csrc/dgp.hip: the survey's scratch constants (one history threshold).
PANEL = DgpParams()
# The tutorial replication (make_tutorial_data): recalibrated to the published run
# (ate_replication.md:118 and the three plots) -- vote-history marginals
# like the real file's (general elections ~0.8, primaries ~0.3-0.45) so the selection
# transform drops ~41,062 of 50,000 rows, and a baseline turnout / effect profile under
# which the published ordering holds: oracle ~0.096, naive ~0, logistic-PS IPW below the
# oracle, LASSO-PS IPW below that, Double ML in [0.03, 0.08] (tools/dgp_calibrate.py,
# tests/test_dgp_calibration.py).
# Thresholds: -Phi^-1(marginal) * sd(history score), marginals (0.85, 0.80, 0.25, 0.40,
# 0.40), sd = sqrt(1 + 0.4^2 (1 + 0.3^2)). At n = 50,000, seed 1991 (CPU reference path,
# tools/dgp_calibrate.py): 40,584 rows dropped (published 41,062), oracle 0.0945 (0.0961),
# naive -0.0012 (0.0028), OLS 0.0888 (0.0777), IPW logistic PS 0.0694 (0.0637), IPW
# LASSO PS 0.0117 (0.0110), Double ML (200 trees) 0.0533 (0.0524).
TUTORIAL = DgpParams(intercept=-1.8, b_hist=(0.35, 0.35, 0.35, 0.35, 0.35), b_latent=0.35,
                     tau_logit=0.4, p_treat=1.0 / 6.0,
                     hist_thresh=(-1.1232, -0.9121, 0.7309, 0.2746, 0.2746), hist_latent=0.4)

# legacy names (the panel model)
INTERCEPT, B_LATENT, TAU_LOGIT, P_TREAT = PANEL.intercept, PANEL.b_latent, PANEL.tau_logit, \
    PANEL.p_treat
B_HIST, HIST_THRESH = PANEL.b_hist[0], PANEL.hist_thresh[0]
HIST_LATENT, YOB_LATENT, FACTOR_LOAD = PANEL.hist_latent, PANEL.yob_latent, PANEL.factor_load


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


def raw_columns(n: int, seed: int, p_extra: int = 0, row_offset: int = 0,
                params: DgpParams = PANEL, idx=None):
    """Unscaled draws for rows [row_offset, row_offset+n), or for the generated-row ids
    ``idx`` (the model of the HIP generator csrc/dgp.hip, row for row; float64 here, float32
    on the device)."""
    P = params
    idx = np.arange(row_offset, row_offset + n, dtype=np.uint64) if idx is None else \
        np.asarray(idx, dtype=np.uint64)
    n = len(idx)
    f = _normal(seed, S_FACTOR, idx)
    fl = P.factor_load
    cts = np.empty((n, 15))
    for j in range(15):
        z = _normal(seed, S_CTS + j, idx)
        cts[:, j] = z if j < 3 else fl * f + np.sqrt(1 - fl ** 2) * z
    latent = _normal(seed, S_LATENT, idx) + P.yob_latent * cts[:, 0]
    hist = np.empty((n, 5))
    for k in range(5):
        hist[:, k] = (_normal(seed, S_HIST + k, idx) + P.hist_latent * latent > P.hist_thresh[k])
    sex = (_uniform(seed, S_SEX, idx) < 0.5).astype(np.float64)
    W = (_uniform(seed, S_W, idx) < P.p_treat).astype(np.float64)
    eta = P.intercept + hist @ np.asarray(P.b_hist, dtype=np.float64) + P.b_latent * latent
    Y = (_uniform(seed, S_Y, idx) < 1.0 / (1.0 + np.exp(-(eta + P.tau_logit * W)))).astype(
        np.float64)
    tau_i = 1 / (1 + np.exp(-(eta + P.tau_logit))) - 1 / (1 + np.exp(-eta))
    extra = np.empty((n, p_extra))
    for j in range(p_extra):
        z = _normal(seed, S_EXTRA + j, idx)
        if j % 4 == 3:   # every 4th extra column is binary
            extra[:, j] = (z > 0).astype(np.float64)
        else:
            extra[:, j] = fl * f + np.sqrt(1 - fl ** 2) * z
    return cts, np.column_stack([sex, hist]), extra, W, Y, tau_i


def selection_flags(seed: int, idx, params: DgpParams, compat: str = "reference") -> np.ndarray:
    """Host twin of csrc/dgp.hip sel_flag for generated rows ``idx``: 1 treated candidate,
    2 control candidate, 0 neither (ate_replication.Rmd:103-110 on the population-
    standardised yob / city, i.e. +-2 on the raw N(0,1) draws; quirk Q17 under
    compat="reference")."""
    P = params
    idx = np.asarray(idx, dtype=np.uint64)
    yob = _normal(seed, S_CTS + 0, idx)
    city = _normal(seed, S_CTS + 1, idx)
    latent = _normal(seed, S_LATENT, idx) + P.yob_latent * yob
    h = [(_normal(seed, S_HIST + k, idx) + P.hist_latent * latent > P.hist_thresh[k])
         for k in range(5)]
    W = _uniform(seed, S_W, idx) < P.p_treat
    last = h[3] if compat == "reference" else h[4]
    dt = h[0] | h[1] | h[2] | h[3] | last | (city > 2) | (yob > 2)
    dc = ~h[0] | ~h[1] | ~h[2] | ~h[3] | ~h[4] | (city < -2) | (yob < -2)
    return np.where(W, np.where(dt, 1, 0), np.where(dc, 2, 0)).astype(np.uint8)


def r_scale(a: np.ndarray) -> np.ndarray:
    """R ``scale()``: centre and divide by the sample SD (n-1 denominator)."""
    m = a.mean(0)
    s = a.std(0, ddof=1)
    s = np.where(s > 0, s, 1.0)
    return (a - m) / s


def make_tutorial_data(n: int = 50_000, seed: int = 1991, p_extra: int = 0,
                       params: DgpParams = TUTORIAL) -> TutorialData:
    """The ``df`` of ``ate_replication.Rmd:89-94`` (scaled cts + binary + Y + W)."""
    cts, binc, extra, W, Y, tau_i = raw_columns(n, seed, p_extra, params=params)
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
