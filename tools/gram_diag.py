"""Where does the paired-tile Gram's time go? Times csrc/gram.hip's pair kernel in three
builds on the N=1e7, p=500 bench panel: normal, GRAM_DIAG=1 (DMA staging + barriers, no
MFMA work) and GRAM_DIAG=2 (MFMA work on stale LDS, no DMA after the prologue).

  python tools/gram_diag.py --build     # here: cross-compile the two timing-only libraries
  python tools/gram_diag.py             # on the GPU box
"""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
LIBS = {m: ROOT / "ate_replication_causalml_amd" / "_lib" / f"libatehip_gdiag{m}.so"
        for m in (1, 2, 3, 4)}


KERNELS = ["pair"]


def build():
    from ate_replication_causalml_amd import _build as B
    B.build_hip()
    objs = [o for o in sorted((ROOT / "build").glob("*.hip.o")) if o.name != "gram.hip.o"]
    for m, lib in LIBS.items():
        o = ROOT / "build" / f"gram_diag{m}.o"
        d = [f"-DGRAM_DIAG={m}"]
        subprocess.run([B.HIPCC, *B.HIP_FLAGS, *d, "-I", str(ROOT / "csrc"), "-c",
                        str(ROOT / "csrc" / "gram.hip"), "-o", str(o)], check=True)
        subprocess.run([B.HIPCC, "-shared", f"--offload-arch={B.ARCH}", "-o", str(lib),
                        *map(str, objs), str(o)], check=True)
        print("built", lib)


def main():
    if "--build" in sys.argv:
        return build()
    n = sys.argv[1] if len(sys.argv) > 1 else "1e7"
    for tag, lib in [("normal", None), ("no-mfma", LIBS[1]), ("no-dma", LIBS[2]),
                     ("no-mfma-offdiag-only", LIBS[3]), ("offdiag-only", LIBS[4])]:
        env = dict(os.environ)
        if lib is not None:
            env["ATE_HIP_LIB"] = str(lib)
        r = subprocess.run([sys.executable, str(ROOT / "tools" / "gram_only.py"), n, *KERNELS],
                           env=env, capture_output=True, text=True, timeout=240)
        for line in r.stdout.strip().splitlines():
            print(f"{tag:8s} rc={r.returncode} {line}", flush=True)
        if r.returncode != 0:
            print(r.stderr[-2000:])
            return r.returncode


if __name__ == "__main__":
    sys.exit(main() or 0)
