#!/bin/bash
set -o pipefail
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_exact" -o ex \
  -- python3 "$ROOT/bench.py" --exact 1 --steps 3 --warmup 1 --parity 0 > "$ROOT/gpurun_out/prof_exact.log" 2>&1 || { echo prof failed; tail -20 "$ROOT/gpurun_out/prof_exact.log"; exit 1; }
echo ok
