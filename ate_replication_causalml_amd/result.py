"""Estimator result record (the ``data.frame(Method, ATE, lower_ci, upper_ci)``
every reference estimator returns, e.g. ``ate_functions.R:20,38,62``) plus an
explicit ``se`` and a diagnostics dict."""
from __future__ import annotations

import json
import math
from dataclasses import asdict, dataclass, field

Z = 1.96  # hard-coded in every reference estimator (ate_functions.R:17-18 etc.)


@dataclass
class AteResult:
    method: str
    ate: float
    se: float                      # NaN when the reference reports no SE (LASSO, Q4)
    lower_ci: float
    upper_ci: float
    diagnostics: dict = field(default_factory=dict)

    @classmethod
    def make(cls, method, ate, se, **diag):
        ate = float(ate)
        if se is None or (isinstance(se, float) and math.isnan(se)):
            return cls(method, ate, float("nan"), ate, ate, diag)
        se = float(se)
        return cls(method, ate, se, ate - Z * se, ate + Z * se, diag)

    def row(self):
        return {"Method": self.method, "ATE": self.ate, "lower_ci": self.lower_ci,
                "upper_ci": self.upper_ci, "se": self.se}

    def to_json(self):
        d = asdict(self)
        d["diagnostics"] = {k: (v if isinstance(v, (int, float, str, bool, type(None))) else str(v))
                            for k, v in d["diagnostics"].items()}
        return json.dumps(d)


def results_frame(results):
    import pandas as pd
    return pd.DataFrame([r.row() for r in results])


def format_table(results) -> str:
    lines = [f"{'Method':45s} {'ATE':>9s} {'SE':>9s} {'lower_ci':>9s} {'upper_ci':>9s}"]
    for r in results:
        se = "" if math.isnan(r.se) else f"{r.se:9.4f}"
        lines.append(f"{r.method:45s} {r.ate:9.4f} {se:>9s} {r.lower_ci:9.4f} {r.upper_ci:9.4f}")
    return "\n".join(lines)
