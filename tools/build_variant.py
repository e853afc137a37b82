"""Build an alternative kernel library for A/B timing: every in-tree object except one
source file, which is recompiled with extra flags.

  python tools/build_variant.py base enet.hip -DENET_BALLOT_ONLY=1
    -> ate_replication_causalml_amd/_lib/libatehip_base.so  (select with ATE_HIP_LIB=...)
  python tools/build_variant.py head build/r/enet.hip@HEAD   (a file written by git show;
    the name before '@' says which in-tree object it replaces)
"""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    name, src, *flags = sys.argv[1:]
    from ate_replication_causalml_amd import _build as B
    B.build_hip()
    path = Path(src) if "/" in src else B.CSRC / src   # a path: e.g. a file from git show
    src = path.name if "/" not in src else src.rsplit("/", 1)[1].split("@")[0]
    objs = [o for o in sorted((ROOT / "build").glob("*.hip.o")) if o.name != src + ".o"]
    vo = ROOT / "build" / f"{Path(src).stem}_{name}.variant.o"
    hip_flags = list(B.HIP_FLAGS)
    if src in B.NO_CONTRACT:
        hip_flags = [f for f in hip_flags if not f.startswith("-ffp-contract")] + ["-ffp-contract=off"]
    subprocess.run([B.HIPCC, *hip_flags, *flags, "-I", str(B.CSRC), "-x", "hip", "-c", str(path),
                    "-o", str(vo)], check=True)
    lib = B.LIBDIR / f"libatehip_{name}.so"
    subprocess.run([B.HIPCC, "-shared", f"--offload-arch={B.ARCH}", "-Wl,-z,defs", "-o", str(lib),
                    *map(str, objs), str(vo)], check=True)
    print("built", lib)


if __name__ == "__main__":
    main()
