"""Structured results logging: the reference prints a data.frame
and three ggplots (ate_replication.Rmd:126-272); here every ``AteResult`` can be
appended to a JSONL file with run metadata, and a results list can be rendered as
the reference's ``geom_pointrange`` comparison plot."""
from __future__ import annotations

import json
import math
import platform
import time


def run_metadata(**extra):
    import torch
    meta = {"time": time.strftime("%Y-%m-%dT%H:%M:%S"), "host": platform.node(),
            "torch": torch.__version__, "hip": getattr(torch.version, "hip", None),
            "gpu": torch.cuda.get_device_name(0) if torch.cuda.is_available() else None}
    meta.update(extra)
    return meta


def write_jsonl(path, results, **meta):
    """Append one JSON line per result (fields of AteResult + run metadata)."""
    m = run_metadata(**meta)
    with open(path, "a") as f:
        for r in results:
            rec = json.loads(r.to_json())
            rec["meta"] = m
            f.write(json.dumps(rec, default=str) + "\n")


def read_jsonl(path):
    with open(path) as f:
        return [json.loads(line) for line in f if line.strip()]


def pointrange_plot(results, path, title=None):
    """ggplot(result_df, aes(y=ATE, x=Method, color=Method)) + geom_pointrange(...)
    (ate_replication.Rmd:145-149,194-198,...)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    fig, ax = plt.subplots(figsize=(max(6, 0.6 * len(results) + 2), 4.5))
    cmap = plt.get_cmap("tab20")
    for i, r in enumerate(results):
        c = cmap(i % 20)
        if not math.isnan(r.se):
            ax.vlines(i, r.lower_ci, r.upper_ci, color=c, lw=1.5)
        ax.plot(i, r.ate, "o", color=c, ms=5)
    ax.set_xticks(range(len(results)))
    ax.set_xticklabels([r.method for r in results], rotation=45, ha="right", fontsize=8)
    ax.set_ylabel("ATE")
    ax.axhline(0.0, color="0.8", lw=0.8, zorder=0)
    if title:
        ax.set_title(title)
    fig.tight_layout()
    fig.savefig(path, dpi=110)
    plt.close(fig)
    return path
