"""The reference's published results: the only fixtures it ships.

* ``ate_replication.md:118``: 41,062 rows dropped by the selection transform;
* ``ate_replication.md:294``: the causal forest's "incorrect" mean-CATE ATE, printed as
  0.083 (SE 0.198);
* ``ate_replication.md:157,233,317``: three pointrange plots, digitised in SURVEY.md §6
  (pixel centroids against the major gridlines; uncertainty about 0.0004 / 0.0005 /
  0.0008 for the three plots). SE = CI half-width / 1.96.

R and the real CSV are absent. The synthetic DGP is calibrated to this table
(data/dgp.py TUTORIAL, tools/dgp_calibrate.py), and ``check_table`` says how a
replication compares with it: rows with a CI must fall inside the published CI
(widened by the digitisation uncertainty); the two LASSO rows, which the reference
prints without a CI (ate_functions.R:107,129), must fall within ``LASSO_BAND`` of the
published point.
"""
from __future__ import annotations

import math

DROPPED = 41_062                 # ate_replication.md:118
DROPPED_REL_TOL = 0.02
CF_MEAN_CATE = (0.083, 0.198)    # ate_replication.md:294: ATE, SE of the mean of CATEs
LASSO_BAND = 0.03
DIGITISE = 0.001                 # >= the largest digitisation uncertainty (0.0008)

# method -> (ATE, lower_ci, upper_ci); lower = upper = ATE for the CI-less LASSO rows
TABLE = {
    "oracle": (0.0961, 0.0850, 0.1073),
    "naive": (0.0028, -0.0238, 0.0294),
    "Direct Method": (0.0777, 0.0520, 0.1034),
    "Propensity_Weighting": (0.0637, 0.0570, 0.0704),
    "Propensity_Regression": (0.0665, 0.0467, 0.0862),
    "Propensity_Weighting_LASSOPS": (0.0110, 0.0076, 0.0145),
    "Single-equation LASSO": (0.0638, 0.0638, 0.0638),
    "Usual LASSO": (0.0249, 0.0249, 0.0249),
    "Doubly Robust with Random Forest PS": (0.0039, -0.0909, 0.0988),
    "Doubly Robust with logistic regression PS": (0.0800, 0.0517, 0.1083),
    "Belloni et.al": (0.0792, 0.0535, 0.1050),
    "Double Machine Learning": (0.0524, 0.0286, 0.0763),
    "residual_balancing": (0.0753, 0.0461, 0.1045),
    "Causal Forest(GRF)": (0.0852, 0.0559, 0.1144),
}
NO_CI = ("Single-equation LASSO", "Usual LASSO")


def check_row(method: str, ate: float, se: float) -> str | None:
    """None if the row agrees with the published one, else a message saying why not."""
    pt, lo, hi = TABLE[method]
    if method in NO_CI:
        if not math.isnan(se):
            return f"{method}: the reference prints no SE (lower_ci = upper_ci), got {se}"
        if abs(ate - pt) > LASSO_BAND:
            return f"{method}: ATE {ate:.4f} not within {LASSO_BAND} of the published {pt}"
        return None
    if not (lo - DIGITISE <= ate <= hi + DIGITISE):
        return f"{method}: ATE {ate:.4f} outside the published CI [{lo}, {hi}]"
    if not (se > 0 and math.isfinite(se)):
        return f"{method}: SE {se} not a positive number"
    return None


def check_table(rows: dict, n_dropped: int | None = None, cf_diag: tuple | None = None) -> list:
    """Every disagreement of a replication with the published table (empty = agrees).
    ``rows``: method -> (ate, se); ``cf_diag``: the causal forest's (mean CATE,
    sqrt(mean var)) diagnostic, compared in sign and magnitude with 0.083 (SE 0.198)."""
    bad = [m for m in TABLE if m not in rows]
    out = [f"missing rows: {bad}"] if bad else []
    for m, (a, s) in rows.items():
        if m in TABLE:
            msg = check_row(m, a, s)
            if msg:
                out.append(msg)
    if n_dropped is not None and abs(n_dropped - DROPPED) > DROPPED_REL_TOL * DROPPED:
        out.append(f"{n_dropped} rows dropped, published {DROPPED} (+-{DROPPED_REL_TOL:.0%})")
    if cf_diag is not None:
        a, s = cf_diag
        pa, ps = CF_MEAN_CATE
        if not (a > 0 and abs(a - pa) <= 0.02):
            out.append(f"causal forest mean CATE {a:.4f}, published {pa} (sign, +-0.02)")
        if not (ps / 2 <= s <= 2 * ps):
            out.append(f"causal forest sqrt(mean var) {s:.4f}, published {ps} (within 2x)")
    return out
