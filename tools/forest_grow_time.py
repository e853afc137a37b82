"""Forest growth time alone (device-binned input): n=1e6 p=100 64 trees and the tutorial
shape n=1e4 p=21 2500 trees (tools/forest_occ.sh)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ate_replication_causalml_amd.models import forest as F  # noqa: E402

dev = torch.device("cuda", 0)
for n, p, nt in [(1_000_000, 100, 64), (10_000, 21, 2500), (1_000_000, 100, 300)]:
    rs = np.random.RandomState(0)
    X = rs.randn(n, p)
    y = (X[:, 0] + 0.5 * X[:, 1] + rs.randn(n) > 0).astype(np.float64)
    Xd = torch.as_tensor(X, device=dev)
    edges = F.bin_edges_device(Xd)
    Xb = F.bin_matrix(Xd, *edges, dev)
    yd = torch.as_tensor(y, device=dev)
    F.fit_forest_binned(Xb, edges, F.KIND_CLASS, y=yd, ntree=4, seed=1)
    torch.cuda.synchronize()
    t = time.perf_counter()
    f = F.fit_forest_binned(Xb, edges, F.KIND_CLASS, y=yd, ntree=nt, seed=1)
    torch.cuda.synchronize()
    nodes = int(f.nnodes.sum()) if hasattr(f, "nnodes") else -1
    print(f"n={n} p={p} trees={nt}: grow {time.perf_counter() - t:.3f}s nodes {nodes}", flush=True)
