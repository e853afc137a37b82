"""Per-row wall time of the 14-row driver on one device: a cold pass (includes
library/kernel-module loading) then warm passes; prints one JSON object."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ate_replication_causalml_amd.api import replicate
from ate_replication_causalml_amd.config import ReplicateConfig, RunConfig
from ate_replication_causalml_amd.data.dgp import make_tutorial_data


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="gpu")
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--n-obs", type=int, default=50000)
    a = ap.parse_args()
    data = make_tutorial_data(a.n_obs, 1991)
    cfg = ReplicateConfig(n_obs=a.n_obs, run=RunConfig(backend=a.backend))
    out = []
    for i in range(a.passes):
        t0 = time.perf_counter()
        rep = replicate(data, cfg)
        total = time.perf_counter() - t0
        out.append({"pass": i, "total_s": total, "rows": {k: round(v, 4) for k, v in rep.seconds.items()}})
        print(json.dumps(out[-1]), flush=True)
    print(json.dumps({"ate": {r.method: [r.ate, r.se] for r in rep.results}}))


if __name__ == "__main__":
    main()
