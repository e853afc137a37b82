"""Phase breakdown of one exact-split tree (csrc/forest_exact.hip built with -DEXACT_PROF).

  python tools/exact_forest_prof.py --build   # here: cross-compile the profiling library
  python tools/exact_forest_prof.py           # on the GPU box: one tree of df_mod, ticks
"""
import ctypes
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
LIB = ROOT / "ate_replication_causalml_amd" / "_lib" / "libatehip_xprof.so"
NAMES = ["setup", "big-node list", "wg decisions", "wave decisions", "ids", "wg partitions",
         "wave partitions", "levels"] + [f"wave{w} busy" for w in range(8)] + [
    "wg stats+draws", "wg key fill", "wg sort", "wg walk+argmax", "wg threshold", "wg nodes"]


def build():
    from ate_replication_causalml_amd import _build as B
    B.build_hip()
    objs = [o for o in sorted((ROOT / "build").glob("*.hip.o")) if o.name != "forest_exact.hip.o"]
    po = ROOT / "build" / "forest_exact_prof.o"
    subprocess.run([B.HIPCC, "-O3", "-fPIC", "-std=c++17", f"--offload-arch={B.ARCH}",
                    "-ffp-contract=off", "-DEXACT_PROF", "-I", str(ROOT / "csrc"), "-c",
                    str(ROOT / "csrc" / "forest_exact.hip"), "-o", str(po)], check=True)
    subprocess.run([B.HIPCC, "-shared", f"--offload-arch={B.ARCH}", "-o", str(LIB),
                    *map(str, objs), str(po)], check=True)
    print("built", LIB)


def run():
    os.environ["ATE_HIP_LIB"] = str(LIB)
    import numpy as np
    import torch
    from ate_replication_causalml_amd import _native
    from ate_replication_causalml_amd.data.dgp import make_tutorial_data
    from ate_replication_causalml_amd.data.selection import apply_selection_bias
    from ate_replication_causalml_amd.models import forest as F
    lib = _native.hip()
    lib.ate_exact_prof_read.argtypes = [ctypes.c_void_p]
    m, _ = apply_selection_bias(make_tutorial_data(50000, 1991), 0.85, 0.85, "reference")
    dev = torch.device("cuda", 0)
    eb = F.exact_bins(m.X)
    Xb = torch.from_numpy(eb.bin(m.X)).to(dev)
    w = torch.as_tensor(m.W, device=dev)
    F.fit_forest_exact(Xb, eb, F.KIND_CLASS, y=w, ntree=1, seed=3)
    torch.cuda.synchronize()
    lib.ate_exact_prof_reset()
    F.fit_forest_exact(Xb, eb, F.KIND_CLASS, y=w, ntree=1, seed=3)
    torch.cuda.synchronize()
    buf = np.zeros(24, dtype=np.uint64)
    lib.ate_exact_prof_read(buf.ctypes.data_as(ctypes.c_void_p))
    for k, v in zip(NAMES, buf):
        print(f"{k:16s} {int(v):10d}" + ("" if k in ("levels", "wg nodes") else f"  ({v / 100:.0f} us)"))


if __name__ == "__main__":
    build() if "--build" in sys.argv else run()
