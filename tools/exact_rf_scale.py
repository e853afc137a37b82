"""The tutorial's randomForest rows at their own tree counts with exact splits on the GPU:
aipw_rf (2500 trees) and double_ml (2000 trees per forest) on df_mod; wall ms of 4 calls
and the ATE bits (for A/B builds selected with ATE_HIP_LIB)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ate_replication_causalml_amd  # noqa: E402,F401
import torch  # noqa: E402

from ate_replication_causalml_amd.data.dgp import make_tutorial_data  # noqa: E402
from ate_replication_causalml_amd.data.selection import apply_selection_bias  # noqa: E402
from ate_replication_causalml_amd.estimators import forest as DF  # noqa: E402

d = make_tutorial_data(50000, 1991)
m, _ = apply_selection_bias(d, 0.85, 0.85, "reference")
dev = torch.device("cuda", 0)
for name, fn in (("aipw_rf", lambda: DF.aipw_rf(m.Y, m.W, m.X, num_trees=2500, device=dev,
                                                 splits="exact")),
                 ("double_ml", lambda: DF.double_ml(m.Y, m.W, m.X, num_trees=2000, device=dev,
                                                    splits="exact"))):
    ts = []
    for _ in range(4):
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    print(f"{os.path.basename(os.environ.get('ATE_HIP_LIB', 'in-tree'))} {name} ms "
          f"{[round(t * 1e3, 1) for t in ts]} ate {r.ate.hex()} se {r.se.hex()}", flush=True)
