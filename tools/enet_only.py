"""Time the CV-LASSO stage of the bench step alone (ops/enet.py:cv_enet_gaussian on the
fold Gram stack of the N=1e7, p=500 bench panel) -- no Gram noise, for A/B of path-kernel
builds: python tools/enet_only.py [reps]   (ATE_HIP_LIB selects an alternative library)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ate_replication_causalml_amd.data.device_dgp import synthetic_panel  # noqa: E402
from ate_replication_causalml_amd.ops.enet import cv_enet_gaussian  # noqa: E402
from ate_replication_causalml_amd.ops.gram import gram  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda", 0)
pan = synthetic_panel(int(1e7), p=500, folds=5, seed=1991, dtype="bf16", device=dev,
                      dgp=os.environ.get("ATE_DGP", "tutorial"))
G = gram(pan).clone()
K = 5
full_sets = [[s for s in range(K) if s != k] for k in range(K)]
ycols = [pan.cols["Y"], pan.cols["W"]]
run = lambda: cv_enet_gaussian(G, pan, pan.xcols, ycols, full_sets=full_sets)  # noqa: E731
for _ in range(2):
    run()
torch.cuda.synchronize()
ts = []
for _ in range(reps):
    e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e[0].record()
    cv = run()
    e[1].record()
    torch.cuda.synchronize()
    ts.append(e[0].elapsed_time(e[1]))
ts.sort()
print(f"enet ms: min {ts[0]:.3f} median {ts[len(ts) // 2]:.3f} max {ts[-1]:.3f}", flush=True)
