"""Cycle breakdown of the CV-LASSO path kernel (csrc/enet.hip built with -DENET_PROF).

  python tools/enet_profile.py --build        # here: cross-compile the profiling library
  python tools/enet_profile.py                # on the GPU box: run one DML step, print
Columns per problem: pull / recurrence / other cycles, block visits, pending columns.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
LIB = ROOT / "ate_replication_causalml_amd" / "_lib" / "libatehip_prof.so"


def build():
    from ate_replication_causalml_amd import _build as B
    B.build_hip()
    objs = sorted((ROOT / "build").glob("*.hip.o"))
    objs = [o for o in objs if o.name not in ("enet.hip.o", "gram.hip.o")]
    prof = []
    for src, flag in (("enet", "-DENET_PROF"), ("gram", "-DGRAM_CLOCK")):
        o = ROOT / "build" / f"{src}_prof.o"
        subprocess.run(B.hip_compile_cmd(ROOT / "csrc" / f"{src}.hip", o) + [flag], check=True)
        prof.append(str(o))
    subprocess.run([B.HIPCC, "-shared", f"--offload-arch={B.ARCH}", "-o", str(LIB),
                    *map(str, objs), *prof], check=True)
    print("built", LIB)


def run(n, p):
    os.environ["ATE_HIP_LIB"] = str(LIB)
    import numpy as np
    import torch
    from ate_replication_causalml_amd import _native
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.lasso import dml_crossfit_panel
    lib = _native.hip()
    lib.ate_enet_prof_read.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    pan = synthetic_panel(n, p=p, folds=5, seed=1991, dtype="bf16", device=dev, dgp=os.environ.get("ATE_DGP", "tutorial"))
    dml_crossfit_panel(pan, 5, "min")
    torch.cuda.synchronize()
    lib.ate_enet_prof_reset()
    t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t[0].record()
    _, _, cv = dml_crossfit_panel(pan, 5, "min")
    t[1].record()
    torch.cuda.synchronize()
    buf = np.zeros((256, 32), dtype=np.uint64)
    lib.ate_enet_prof_read(buf.ctypes.data_as(ctypes.c_void_p))
    rows = buf[:40]
    live = rows[rows[:, 3] > 0]
    print(json.dumps({"step_ms": t[0].elapsed_time(t[1]),
                      "per_problem": [[int(v) for v in r[:32]] for r in live],
                      "note": "[0] phase B + pass-start pulls, [1] phase A, [2] wave-0 phase A, [3] visits, [4] wave-1 phase A, [5] wall ticks inside passes, [6] wave-0 loop ticks, [7] updates, [8] pass-start pulls, [9] wave-0 phase B, [10] shader cycles, [11] wall ticks (100 MHz), [12] mode-L passes with visits, [13] empty passes, [14] wave-0 visits, [15] loop-only cycles, [16] wave-1 phase B, [17] prologue cycles, [18] last pull wave phase A, [19]-[22] mode S passes / candidates / cycles / fetches, [23] mode-S loop cycles, [24] prologue before the arrival wait, [25] the wait, [26] after the wait, [27] wave-0 phase-A barrier, [28] post-walk cycles"}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--p", type=int, default=500)
    a = ap.parse_args()
    if a.build:
        build()
    else:
        run(a.rows, a.p)
