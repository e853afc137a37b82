#!/bin/bash
# One GPU-box pass: gpu tests, smoke, bench, kernel profile of the bench.
set -o pipefail
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_bench" -o bench \
  -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 > "$ROOT/gpurun_out/prof_bench.log" 2>&1 || { echo prof failed; exit 1; }

python3 -c "import sys; sys.path.insert(0, '$ROOT/tools'); import timeline; timeline.overlapped(sys.argv[1], 24)" $(find $ROOT/gpurun_out/prof_bench -name "*kernel_trace.csv") > $ROOT/gpurun_out/prof_bench_timeline.txt 2>&1 || true
echo done
