"""Residual balancing (E14) on the tutorial df_mod, called 4 times (eager, capture, two
replays) for a kernel profile: rocprofv3 --kernel-trace --stats -- python3 tools/arb_profile.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ate_replication_causalml_amd  # noqa: E402,F401
import torch  # noqa: E402

from ate_replication_causalml_amd.data.dgp import make_tutorial_data  # noqa: E402
from ate_replication_causalml_amd.data.selection import apply_selection_bias  # noqa: E402
from ate_replication_causalml_amd.estimators.balance import residual_balance  # noqa: E402

d = make_tutorial_data(50000, 1991)
m, _ = apply_selection_bias(d, 0.85, 0.85, "reference")
graph = len(sys.argv) < 2 or sys.argv[1] != "eager"
for i in range(int(os.environ.get("REPS", "4"))):
    t0 = time.perf_counter()
    r = residual_balance(m.Y, m.W, m.X, device=torch.device("cuda", 0), graph=graph)
    torch.cuda.synchronize()
    print(i, round(time.perf_counter() - t0, 4), r.ate, r.diagnostics, flush=True)
