#!/bin/bash
# Round-6: exact-forest overflow check moved to the first host read -- forest GPU tests,
# config-4 phases and three config-4 timings
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local n=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$n.log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] failed rc=$rc"; tail -30 "$OUT/$n.log"; exit $rc; fi
  echo "[$n] ok: $(tail -1 "$OUT/$n.log" | cut -c1-300)"; }
step tests 600 python -u -m pytest tests/test_forest_gpu.py tests/test_gpu_graph_estimators.py -x -q --timeout 240 --timeout-method thread
step phases 300 python -u tools/cfg4_phases.py
for i in 1 2 3; do step cfg4_$i 200 python -u tools/bench_configs.py --configs 4; done
