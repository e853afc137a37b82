"""Race/memory-safety checks of the host C++ code: the forest engine (binned
and exact-split trees, every sampling mode, both predictors, the variance debiaser)
built with AddressSanitizer + UndefinedBehaviorSanitizer (GPU sanitizers are not
available on this pool; the GPU kernels are instead checked bit-for-bit against this
engine in tests/test_forest_gpu.py)."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_forest_engine_asan_ubsan(tmp_path):
    exe = tmp_path / "forest_asan"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fopenmp",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-ffp-contract=off",
           "-I", str(ROOT / "csrc"), str(ROOT / "tests" / "native" / "forest_asan_main.cpp"),
           str(ROOT / "csrc" / "cpu" / "forest_cpu.cpp"), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1", OMP_NUM_THREADS="2")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
    assert r.stdout.count(" ok:") == 9
