"""A/B of the single ate_dml call (bench.py's timed step) over Gram kernels on ONE panel:
the panel is generated once, each variant's step is captured and timed in alternation
(K calls back to back, R rounds), so box-to-box and clock drift cancel out.
Usage: single_ab.py [tri,pair] [rounds] [calls]   (variants: tri | pair | pair16, with an
optional @rN suffix: the paired Gram's plan built for N whole rounds of workgroups)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ate_replication_causalml_amd.data.device_dgp import synthetic_panel  # noqa: E402
from ate_replication_causalml_amd.data import device_dgp  # noqa: E402

device_dgp.BYTE_PANEL = True      # the byte copy, so that pair / pair16 A/B both run
from ate_replication_causalml_amd.estimators.lasso import dml_phases, global_seg_counts  # noqa: E402
from ate_replication_causalml_amd.ops import gram as gram_mod  # noqa: E402
from ate_replication_causalml_amd.parallel.comm import LocalComm  # noqa: E402
from ate_replication_causalml_amd.utils.graphs import SegmentedStep  # noqa: E402

variants = (sys.argv[1] if len(sys.argv) > 1 else "tri,pair").split(",")
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 20
dev = torch.device("cuda", 0)
pan = synthetic_panel(int(1e7), p=500, folds=5, seed=1991, dtype="bf16", blocked=True, device=dev,
                      dgp=os.environ.get("ATE_DGP", "tutorial"))
seg = global_seg_counts(pan, LocalComm())
steps = {}
def _select(v):
    v, _, r = v.partition("@r")
    gram_mod.GRAM_TRI = v == "tri"
    gram_mod.BYTE_COLS = v != "pair16"      # pair16: the byte columns read as bf16
    if r:
        os.environ["ATE_GRAM_ROUNDS"] = r
    else:
        os.environ.pop("ATE_GRAM_ROUNDS", None)


for i, v in enumerate(variants):
    _select(v)
    with gram_mod.plan_slot(10 + i):
        steps[v] = SegmentedStep(dml_phases(pan, 5, "min", seg_counts=seg), graph=True)
times = {v: [] for v in variants}
res = {}
for r in range(rounds):
    for v in variants:
        _select(v)      # the captured steps launch with their own settings; eager kept in sync
        for _ in range(3):
            steps[v]()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(calls):
            out = steps[v]()
        torch.cuda.synchronize()
        times[v].append((time.perf_counter() - t0) / calls * 1e3)
        res[v] = [float(x).hex() for x in out["res"].cpu()]
for v in variants:
    t = sorted(times[v])
    print(f"{v}: ms/call median {t[len(t) // 2]:.3f} all {[round(x, 3) for x in times[v]]} "
          f"res {res[v]}", flush=True)
