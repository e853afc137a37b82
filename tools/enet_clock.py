"""Shader clock of the CV path kernel alone vs beside a running Gram (DVFS under load):
the profiling build's per-problem clock64 / wall_clock64 deltas ([10] / [11], csrc/enet.hip
ENET_PROF) give each problem's average clock. Also the wall time of the path launch. Then
the Gram tile kernel's own clock (csrc/gram.hip GRAM_CLOCK: per-workgroup clock64 /
wall_clock64) alone and beside path launches on another stream.

  python tools/enet_profile.py --build     # here: the profiling library
  python tools/enet_clock.py               # GPU box
"""
import ctypes
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
os.environ["ATE_HIP_LIB"] = str(ROOT / "ate_replication_causalml_amd" / "_lib" / "libatehip_prof.so")


def main():
    import numpy as np
    import torch
    from ate_replication_causalml_amd import _native
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.lasso import dml_crossfit_panel
    from ate_replication_causalml_amd.ops import gram as G
    lib = _native.hip()
    lib.ate_enet_prof_read.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    pan = synthetic_panel(10_000_000, p=500, folds=5, seed=1991, dtype="bf16", device=dev, dgp=os.environ.get("ATE_DGP", "tutorial"))
    Gs = G.gram(pan)
    torch.cuda.synchronize()
    from ate_replication_causalml_amd.ops.enet import cv_enet_gaussian
    K = 5
    full_sets = [[s for s in range(K) if s != k] for k in range(K)]
    ycols = [pan.cols["Y"], pan.cols["W"]]

    def path():
        return cv_enet_gaussian(Gs, pan, pan.xcols, ycols, full_sets=full_sets)

    path()
    torch.cuda.synchronize()
    side = torch.cuda.Stream(priority=0)
    out = {}
    for mode in ("alone", "beside_gram", "alone"):
        lib.ate_enet_prof_reset()
        if mode == "beside_gram":
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(3):
                    G.gram(pan, stage="tiles")
        e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e[0].record()
        path()
        e[1].record()
        torch.cuda.synchronize()
        buf = np.zeros((256, 32), dtype=np.uint64)
        lib.ate_enet_prof_read(buf.ctypes.data_as(ctypes.c_void_p))
        live = buf[buf[:, 11] > 0]
        ghz = live[:, 10].astype(float) / live[:, 11].astype(float) * 0.1
        out.setdefault(mode, []).append({"path_ms": round(e[0].elapsed_time(e[1]), 3),
                                         "clock_ghz_median": round(float(np.median(ghz)), 3),
                                         "clock_ghz_min": round(float(ghz.min()), 3),
                                         "clock_ghz_max": round(float(ghz.max()), 3)})
    # the Gram tile kernel's own clock (GRAM_CLOCK build): alone, and beside path launches
    lib.ate_gram_clock_read.argtypes = [ctypes.c_void_p]
    for mode in ("gram_alone", "gram_beside_path", "gram_alone"):
        torch.cuda.synchronize()
        lib.ate_gram_clock_reset()
        if mode == "gram_beside_path":
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(4):
                    path()
        e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e[0].record()
        for _ in range(3):
            G.gram(pan, stage="tiles")
        e[1].record()
        torch.cuda.synchronize()
        gc = np.zeros(3, dtype=np.uint64)
        lib.ate_gram_clock_read(gc.ctypes.data_as(ctypes.c_void_p))
        out.setdefault(mode, []).append({
            "gram_ms": round(e[0].elapsed_time(e[1]) / 3, 3),
            "clock_ghz_mean": round(float(gc[0]) / max(float(gc[1]), 1.0) * 0.1, 3),
            "workgroups": int(gc[2])})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
