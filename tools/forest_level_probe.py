"""One config-3 forest on the level engine vs the per-tree kernel: the propensity forest of
fold 0 of the per-GPU shard (N=1e7 panel, p=500, 8e6 training rows, 13 trees), phase
timing with ATE_FOREST_LV_PROF=1. Prints one line per engine."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ate_replication_causalml_amd  # noqa: E402,F401


def main():
    import torch
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.boosting import bin_panel
    from ate_replication_causalml_amd.models import forest as F
    n = int(float(os.environ.get("N", "1e7")))
    trees = int(os.environ.get("TREES", "13"))
    dev = torch.device("cuda", 0)
    pan = synthetic_panel(n, p=500, folds=5, seed=11, dtype="bf16", device=dev)
    Xr, ldr, edges, rows = bin_panel(pan)
    Xb = Xr[:, :500].t().contiguous()
    del Xr
    W = pan.col("W").index_select(0, rows).double()
    nr = pan.seg_nreal
    a = int(nr[0])
    idx = torch.arange(a, Xb.shape[1], device=dev)
    Xt = Xb.index_select(1, idx)
    yt = W.index_select(0, idx)
    del pan
    for eng in os.environ.get("ENGINES", "level,tree").split(","):
        os.environ["ATE_FOREST_ENGINE"] = eng
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fr = F.fit_forest_binned(Xt, edges, F.KIND_CLASS, y=yt, ntree=trees, seed=1991 + 1000)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        nn = fr.nnodes.cpu()
        print(json.dumps({"engine": eng, "n_train": Xt.shape[1], "trees": trees, "seconds": dt,
                          "nodes_tree0": int(nn[0]), "nodes_sum": int(nn.sum())}), flush=True)
        del fr


if __name__ == "__main__":
    main()
