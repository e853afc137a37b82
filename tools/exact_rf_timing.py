"""aipw_rf / double_ml on the tutorial df_mod: exact-split vs 256-bin forests on the GPU
(graph replays after a capture) and on the host twin; ATE / SE / wall time per call."""
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
print("n", len(m.Y), flush=True)
for splits in ("exact", "binned"):
    for name, fn in (("aipw_rf", lambda dev: DF.aipw_rf(m.Y, m.W, m.X, num_trees=100, device=dev,
                                                        splits=splits)),
                     ("double_ml", lambda dev: DF.double_ml(m.Y, m.W, m.X, num_trees=100,
                                                            device=dev, splits=splits))):
        ts = []
        for _ in range(4):
            t0 = time.perf_counter()
            r = fn(torch.device("cuda", 0))
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        c = fn("cpu")
        tc = time.perf_counter() - t0
        print(f"{splits:6s} {name:9s} gpu ate {r.ate:.10f} se {r.se:.10f} graph "
              f"{r.diagnostics.get('hipgraph')} ms {[round(t * 1e3, 1) for t in ts]} | cpu ate "
              f"{c.ate:.10f} se {c.se:.10f} ms {tc * 1e3:.0f}", flush=True)
