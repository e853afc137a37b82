"""Phase split of the forest growth kernel (csrc/forest.hip built with -DFOREST_PROF).

  python tools/forest_profile.py --build      # here: cross-compile the profiling library
  python tools/forest_profile.py             # on the GPU box: grow one RF, print per-tree means
Columns: decisions / child ids / partition / setup (ms, wall_clock64 at 100 MHz), levels,
nodes, nodes <= 16 rows, nodes of 17-64 rows.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
LIB = ROOT / "ate_replication_causalml_amd" / "_lib" / "libatehip_fprof.so"


def build():
    from ate_replication_causalml_amd import _build as B
    B.build_hip()
    objs = [o for o in sorted((ROOT / "build").glob("*.hip.o")) if o.name != "forest.hip.o"]
    po = ROOT / "build" / "forest_prof.o"
    subprocess.run([B.HIPCC, "-O3", "-fPIC", "-std=c++17", f"--offload-arch={B.ARCH}",
                    "-ffp-contract=off", "-DFOREST_PROF", "-I", str(ROOT / "csrc"), "-c",
                    str(ROOT / "csrc" / "forest.hip"), "-o", str(po)], check=True)
    subprocess.run([B.HIPCC, "-shared", f"--offload-arch={B.ARCH}", "-o", str(LIB),
                    *map(str, objs), str(po)], check=True)
    print("built", LIB)


def run(n, p, trees):
    os.environ["ATE_HIP_LIB"] = str(LIB)
    import numpy as np
    import torch
    from ate_replication_causalml_amd import _native
    from ate_replication_causalml_amd.models import forest as F
    lib = _native.hip()
    lib.ate_forest_prof_read.argtypes = [ctypes.c_void_p]
    rs = np.random.RandomState(0)
    X = rs.randn(n, p)
    y = (X[:, 0] + 0.5 * X[:, 1] + rs.randn(n) > 0).astype(float)
    F.fit_forest(X, F.KIND_CLASS, y=y, ntree=4, seed=1, backend="gpu")
    torch.cuda.synchronize()
    lib.ate_forest_prof_reset()
    t0 = time.perf_counter()
    F.fit_forest(X, F.KIND_CLASS, y=y, ntree=trees, seed=1, backend="gpu")
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    buf = np.zeros((1024, 8), dtype=np.uint64)
    lib.ate_forest_prof_read(buf.ctypes.data_as(ctypes.c_void_p))
    rows = buf[:trees].astype(float)
    m = rows.mean(0)
    print(json.dumps({"wall_s": wall, "trees": trees, "n": n, "p": p,
                      "ms": {"decisions": m[0] / 1e5, "child_ids": m[1] / 1e5,
                             "partition": m[2] / 1e5, "setup": m[7] / 1e5},
                      "levels": m[3], "nodes": m[4], "nodes_le16": m[5], "nodes_17_64": m[6]}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--n", type=int, default=160_000)
    ap.add_argument("--p", type=int, default=100)
    ap.add_argument("--trees", type=int, default=100)
    a = ap.parse_args()
    if a.build:
        build()
    else:
        run(a.n, a.p, a.trees)
