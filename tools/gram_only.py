"""Run the bf16 Gram kernel alone on the N=1e7, p=500 bench panel (for PMC profiling)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ate_replication_causalml_amd.data.device_dgp import synthetic_panel  # noqa: E402
from ate_replication_causalml_amd.ops.gram import gram  # noqa: E402

pan = synthetic_panel(int(float(sys.argv[1]) if len(sys.argv) > 1 else 1e7), p=500, folds=5,
                      seed=1991, dtype="bf16", device=torch.device("cuda", 0))
for _ in range(3):
    gram(pan)
torch.cuda.synchronize()
e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e[0].record()
for _ in range(5):
    gram(pan)
e[1].record()
torch.cuda.synchronize()
print("gram ms", e[0].elapsed_time(e[1]) / 5)
