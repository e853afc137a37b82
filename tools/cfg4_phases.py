"""Config 4 phase timing (causal forest 2000 trees + 1000 bootstrap reps, tutorial DGP,
n=5e4 p=21): the two orthogonalisation forests, their OOB predictions, the causal forest,
its OOB prediction and the bootstrap, for exact (grf default at this size) and binned
splits. One warm-up pass per mode, then a timed pass. Prints one JSON line per mode.

    python tools/cfg4_phases.py [n]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ate_replication_causalml_amd  # noqa: E402,F401


def main():
    import numpy as np
    import torch
    from ate_replication_causalml_amd.data.dgp import make_tutorial_data
    from ate_replication_causalml_amd.models import forest as F
    from ate_replication_causalml_amd.estimators.linear import bootstrap_replicates  # noqa: F401
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 50000
    d = make_tutorial_data(n, seed=12)
    X, Y, W = (np.asarray(a, dtype=np.float64) for a in (d.X, d.Y, d.W))
    dev = torch.device("cuda", 0)

    def sync():
        torch.cuda.synchronize()

    modes = os.environ.get("MODES", "exact,binned,exact,binned").split(",")
    for splits in modes:
        t = {}
        sync()
        t0 = time.perf_counter()
        nt = 500
        p = X.shape[1]
        edges = F.exact_bins(X) if splits == "exact" else F.bin_edges(X)
        grf = dict(mtry=F.grf_mtry(p), min_node=5, sampling=1, honesty=True, mtry_poisson=True,
                   alpha=0.05, sample_fraction=0.5, backend="gpu", edges=edges, splits=splits)
        t["bins"] = time.perf_counter() - t0
        t1 = time.perf_counter()
        fy = F.fit_forest(X, F.KIND_REG, r1=Y, ntree=nt, seed=12346, group=1, **grf)
        fw = F.fit_forest(X, F.KIND_REG, r1=W, ntree=nt, seed=12347, group=1, **grf)
        sync()
        t["nuisance_fit"] = time.perf_counter() - t1
        t1 = time.perf_counter()
        y_hat = fy.predict_raw(None, oob=True)
        w_hat = fw.predict_raw(None, oob=True)
        t["nuisance_oob"] = time.perf_counter() - t1
        t1 = time.perf_counter()
        fc = F.fit_forest(X, F.KIND_CAUSAL, r1=W - w_hat, r2=Y - y_hat, ntree=2000, seed=12345,
                          group=2, **grf)
        sync()
        t["causal_fit"] = time.perf_counter() - t1
        t1 = time.perf_counter()
        out = fc.predict_raw(None, oob=True)
        t["causal_oob"] = time.perf_counter() - t1
        t["total"] = time.perf_counter() - t0
        t["nodes_causal"] = int(np.asarray(fc.nnodes.cpu() if hasattr(fc.nnodes, "cpu") else fc.nnodes).sum())
        print(json.dumps({"splits": splits, "n": n, **{k: round(v, 4) if isinstance(v, float) else v
                                                      for k, v in t.items()},
                          "tau_mean": float(np.nanmean(out[:, 0]))}), flush=True)


if __name__ == "__main__":
    main()
