"""Exact-split forest growth alone on the GPU (df_mod shape): kernel time vs trees and
node size, to see where a tree's time goes (latency of one tree vs 100 in parallel)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ate_replication_causalml_amd  # noqa: E402,F401
import torch  # noqa: E402

from ate_replication_causalml_amd.data.dgp import make_tutorial_data  # noqa: E402
from ate_replication_causalml_amd.data.selection import apply_selection_bias  # noqa: E402
from ate_replication_causalml_amd.models import forest as F  # noqa: E402

d = make_tutorial_data(50000, 1991)
m, _ = apply_selection_bias(d, 0.85, 0.85, "reference")
X, W = m.X, m.W
dev = torch.device("cuda", 0)
eb = F.exact_bins(X)
Xb = torch.from_numpy(eb.bin(X)).to(dev)
de = eb.on(dev)
w = torch.as_tensor(W, device=dev)
print("n", X.shape, "distinct per feature", eb.nval.tolist(), flush=True)
for splits in ("exact", "binned"):
    if splits == "binned":
        edges = F.bin_edges(X)
        Xb8 = F.bin_matrix(X, *edges, dev)
    for ntree in (1, 8, 100, 500):
        for mn in (1, 5):
            for rep in range(2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                if splits == "exact":
                    fr = F.fit_forest_exact(Xb, de, F.KIND_CLASS, y=w, ntree=ntree, seed=3,
                                            min_node=mn)
                else:
                    fr = F.fit_forest_binned(Xb8, (None, None), F.KIND_CLASS, y=w, ntree=ntree,
                                             seed=3, min_node=mn)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
            nn = fr.nnodes.cpu().numpy()
            print(f"{splits:6s} ntree {ntree:4d} min_node {mn} ms {dt * 1e3:8.2f} "
                  f"nodes/tree {nn.mean():.0f}", flush=True)
