#!/bin/bash
# Round-6 error-legibility session: (1) the round-5 r05_s3 failure re-run on that tree
# (_r5s3: commit 357f8a4 with the launch-error machinery backported) on its debug library;
# (2) the named invalid-launch test on the production and debug libraries; (3) the GPU
# suite on the debug library (load-time kernel resource check).
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
( cd _r5s3 && ATE_DEBUG=1 timeout -k 10 300 python -u -m pytest tests/test_forest_gpu.py -x -v \
    --timeout 200 --timeout-method thread -k test_device_forest_estimators_match_host \
    > "$ROOT/$OUT/r5s3_repro.log" 2>&1 ); rc=$?
echo "[r5s3_repro] rc=$rc"; grep -E "failed with status|passed|failed" "$OUT/r5s3_repro.log" | tail -5
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step() { local n=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$n.log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] failed rc=$rc"; tail -30 "$OUT/$n.log"; exit $rc; fi
  echo "[$n] ok: $(tail -1 "$OUT/$n.log" | cut -c1-300)"; }
step named 200 python -u -m pytest tests/test_gpu.py -x -v -s --timeout 120 --timeout-method thread -k invalid_launch
ATE_DEBUG=1 step named_debug 200 python -u -m pytest tests/test_gpu.py -x -v -s --timeout 120 --timeout-method thread -k invalid_launch
ATE_DEBUG=1 step debugtests 1200 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
step tests_sel 300 python -u -m pytest tests/test_gpu_panel_selection.py -x -v --timeout 200 --timeout-method thread
step bench 400 python -u bench.py
