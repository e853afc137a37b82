"""In-tree build of the native libraries.

* ``_lib/libatehip.so`` — every ``csrc/*.hip`` file compiled for gfx950 with hipcc
  (cross-compiles without a GPU) and linked into one shared object.
* ``_lib/libatecpu.so`` — host C++ (``csrc/cpu/*.cpp``): CPU forest engine used by
  the float64 reference path and as a host runtime.

Usage: ``python -m ate_replication_causalml_amd._build`` (or ``__graft_entry__.build()``).
Object files are cached under ``build/`` keyed by source mtime.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
LIBDIR = Path(__file__).resolve().parent / "_lib"
BUILD = ROOT / "build"
ARCH = os.environ.get("ATE_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

HIP_FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-ffp-contract=fast-honor-pragmas", "-Wno-unused-result"]
NO_CONTRACT = {"forest.hip", "forest_level.hip", "forest_exact.hip", "gbdt.hip"}
CPU_FLAGS = ["-O3", "-fPIC", "-std=c++17", "-fopenmp", "-ffp-contract=off", "-march=x86-64-v2"]


def _headers(d: Path):
    return [p for p in d.glob("*.hpp")] + [p for p in d.glob("*.h")]


def _stale(obj: Path, deps) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(p.stat().st_mtime > t for p in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(map(str, cmd))}\n{r.stdout}\n{r.stderr}")
    return r


DEBUG_FLAGS = ["-DATE_DEVICE_ASSERT"]   # device bounds checks (csrc/common.hpp ATE_DASSERT)


def debug_enabled() -> bool:
    """``ATE_DEBUG=1``: build / load the device-assertion library (libatehip_debug.so)."""
    return os.environ.get("ATE_DEBUG", "0") not in ("", "0")


def hip_compile_cmd(src: Path, obj: Path, debug: bool = False) -> list:
    """hipcc command line of one kernel source (``debug``: with the device assertions)."""
    flags = list(HIP_FLAGS)
    if src.name in NO_CONTRACT:
        # bit-exact parity with the host reference: no FMA contraction
        flags = [f for f in flags if not f.startswith("-ffp-contract")] + ["-ffp-contract=off"]
    if debug:
        flags += DEBUG_FLAGS
    return [HIPCC, *flags, "-I", str(CSRC), "-c", str(src), "-o", str(obj)]


def hip_lib_name(debug: bool = False) -> str:
    return "libatehip_debug.so" if debug else "libatehip.so"


def build_hip(verbose: bool = False, debug: bool | None = None) -> Path:
    """Compile every csrc/*.hip for gfx950 and link _lib/libatehip.so; ``debug`` (default:
    ATE_DEBUG) builds the device-assertion variant into build/debug/ and
    _lib/libatehip_debug.so instead (the production library is untouched)."""
    debug = debug_enabled() if debug is None else debug
    srcs = sorted(CSRC.glob("*.hip"))
    hdrs = _headers(CSRC)
    bdir = BUILD / "debug" if debug else BUILD
    bdir.mkdir(parents=True, exist_ok=True)
    LIBDIR.mkdir(exist_ok=True)
    objs = []
    jobs = []
    for s in srcs:
        o = bdir / (s.stem + ".hip.o")
        objs.append(o)
        if _stale(o, [s, *hdrs, Path(__file__)]):
            jobs.append(hip_compile_cmd(s, o, debug))
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        list(ex.map(_run, jobs))
    lib = LIBDIR / hip_lib_name(debug)
    if jobs or not lib.exists():
        _run([HIPCC, "-shared", f"--offload-arch={ARCH}", "-Wl,-z,defs", "-o", str(lib), *map(str, objs)])
    if verbose:
        print(f"built {lib} ({len(jobs)} recompiled)")
    return lib


def build_cpu(verbose: bool = False) -> Path:
    cdir = CSRC / "cpu"
    srcs = sorted(cdir.glob("*.cpp"))
    LIBDIR.mkdir(exist_ok=True)
    lib = LIBDIR / "libatecpu.so"
    if not srcs:
        return lib
    deps = [*srcs, *_headers(cdir), *_headers(CSRC), Path(__file__)]
    if _stale(lib, deps):
        _run(["g++", *CPU_FLAGS, "-I", str(CSRC), "-shared", "-o", str(lib), *map(str, srcs)])
    if verbose:
        print(f"built {lib}")
    return lib


def build_all(verbose: bool = False):
    """The production kernel library, the host library and the device-assertion kernel
    library (_lib/libatehip_debug.so, loaded with ATE_DEBUG=1): both kernel libraries are
    rebuilt from the same sources, so the debug build is never older than the production
    one (ATE_NO_DEBUG_BUILD=1 skips it)."""
    out = (build_hip(verbose, debug=False), build_cpu(verbose))
    if os.environ.get("ATE_NO_DEBUG_BUILD", "0") in ("", "0"):
        build_hip(verbose, debug=True)
    return out


if __name__ == "__main__":
    build_all(verbose=True)
    sys.exit(0)
