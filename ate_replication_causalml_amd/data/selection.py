"""Selection-bias transform of ``ate_replication.Rmd:97-121`` (P7, quirks Q17/Q18).

Treated "likely voters" and control "unlikely voters" are dropped: for each arm
the FIRST ``round(0.85 * k)`` matching rows in row order are removed (not a
random 85%). The treated rule repeats ``p2002`` and omits ``p2004``
(``ate_replication.Rmd:104``) — reproduced verbatim under
``compat="reference"``; ``compat="textbook"`` uses ``p2004``.
"""
from __future__ import annotations

import numpy as np


def r_round(x: float) -> int:
    """R's round(): IEC 60559 round-half-even."""
    return int(np.round(x))


def selection_masks(X: np.ndarray, names, compat: str = "reference"):
    col = {n: X[:, i] for i, n in enumerate(names)}
    last = "p2002" if compat == "reference" else "p2004"
    drop_treat = ((col["g2000"] == 1) | (col["g2002"] == 1) |
                  (col["p2000"] == 1) | (col["p2002"] == 1) | (col[last] == 1) |
                  (col["city"] > 2) | (col["yob"] > 2))
    drop_control = ((col["g2000"] == 0) | (col["g2002"] == 0) |
                    (col["p2000"] == 0) | (col["p2002"] == 0) | (col["p2004"] == 0) |
                    (col["city"] < -2) | (col["yob"] < -2))
    return drop_treat, drop_control


def drop_indices(X, W, names, pt: float = 0.85, pc: float = 0.85, compat: str = "reference"):
    """Row indices removed by the transform (the printed ``length(drop_idx)``)."""
    dt, dc = selection_masks(X, names, compat)
    treat_idx = np.flatnonzero((W == 1) & dt)
    ctrl_idx = np.flatnonzero((W == 0) & dc)
    # R: x[1:round(p*k)] ; with k == 0 R's 1:0 would yield c(1, 0) -> index 1; guard it.
    kt = r_round(pt * len(treat_idx))
    kc = r_round(pc * len(ctrl_idx))
    return np.unique(np.concatenate([treat_idx[:kt], ctrl_idx[:kc]]))


def apply_selection_bias(data, pt: float = 0.85, pc: float = 0.85, compat: str = "reference"):
    """Return (df_mod data, dropped indices)."""
    from .dgp import TutorialData
    drop = drop_indices(data.X, data.W, data.names, pt, pc, compat)
    keep = np.ones(data.n, dtype=bool)
    keep[drop] = False
    mod = TutorialData(X=data.X[keep], W=data.W[keep], Y=data.Y[keep], names=list(data.names),
                       tau_true=data.tau_true)
    return mod, drop
