"""Exact-mode Gram vs the default Gram on the bench panel (N=1e7, p=500, bf16, blocked):
tile kernel and reduce timed separately with HIP events."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ate_replication_causalml_amd  # noqa: E402,F401
import torch  # noqa: E402

from ate_replication_causalml_amd.data.device_dgp import synthetic_panel  # noqa: E402
from ate_replication_causalml_amd.estimators.lasso import EXACT_BLOCK  # noqa: E402
from ate_replication_causalml_amd.ops.gram import gram  # noqa: E402

dev = torch.device("cuda", 0)
blk = int(os.environ.get("BLOCK", EXACT_BLOCK))
pan = synthetic_panel(int(1e7), p=500, folds=5, seed=1991, dtype="bf16", blocked=True, device=dev,
                      align=blk)


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for ex in (False, True):
    t = timed(lambda: gram(pan, stage="tiles", exact=ex))
    r = timed(lambda: gram(pan, stage="reduce", exact=ex))
    from ate_replication_causalml_amd.ops.gram import plan_for
    pl = plan_for(pan, exact=ex)
    print(f"exact={ex} block={blk} chunks={os.environ.get('ATE_GRAM_EXACT_CHUNKS', '')} "
          f"nchunks={pl.nchunks} ntiles={pl.ntiles} tiles {t:.3f} ms reduce {r:.3f} ms",
          flush=True)
