"""Phase breakdown of one exact-split tree (csrc/forest_exact.hip built with -DEXACT_PROF).

  python tools/exact_forest_prof.py --build   # here: cross-compile the profiling library
  python tools/exact_forest_prof.py           # on the GPU box: one tree of df_mod, ticks
  python tools/exact_forest_prof.py --causal  # ... tree 0 of a config-4 grf causal forest
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
    dev = torch.device("cuda", 0)
    if "--causal" in sys.argv:
        # one grf causal tree of config 4 (n=5e4, p=21: little bags, honesty, Poisson mtry 21)
        d = make_tutorial_data(50000, seed=12)
        X = np.asarray(d.X, dtype=np.float64)
        eb = F.exact_bins(X)
        Xb = torch.from_numpy(eb.bin(X, grf=True)).to(dev)
        Wc = np.asarray(d.W, dtype=np.float64)
        Yc = np.asarray(d.Y, dtype=np.float64)
        kw = dict(r1=Wc - Wc.mean(), r2=Yc - Yc.mean(), ntree=2, mtry=F.grf_mtry(X.shape[1]),
                  min_node=5, sampling=1, honesty=True, group=2, mtry_poisson=True, alpha=0.05,
                  sample_fraction=0.5, seed=12345)
        fit = lambda: F.fit_forest_exact(Xb, eb, F.KIND_CAUSAL, **kw)
    else:
        m, _ = apply_selection_bias(make_tutorial_data(50000, 1991), 0.85, 0.85, "reference")
        eb = F.exact_bins(m.X)
        Xb = torch.from_numpy(eb.bin(m.X)).to(dev)
        w = torch.as_tensor(m.W, device=dev)
        fit = lambda: F.fit_forest_exact(Xb, eb, F.KIND_CLASS, y=w, ntree=1, seed=3)
    fit()
    torch.cuda.synchronize()
    lib.ate_exact_prof_reset()
    fit()
    torch.cuda.synchronize()
    buf = np.zeros(24, dtype=np.uint64)
    lib.ate_exact_prof_read(buf.ctypes.data_as(ctypes.c_void_p))
    for k, v in zip(NAMES, buf):
        print(f"{k:16s} {int(v):10d}" + ("" if k in ("levels", "wg nodes") else f"  ({v / 100:.0f} us)"))


if __name__ == "__main__":
    build() if "--build" in sys.argv else run()
