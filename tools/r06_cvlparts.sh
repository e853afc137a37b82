#!/bin/bash
# Round-6: CV-loss rows split over ATE_CVL_PARTS workgroups per (problem, lambda chunk):
# GPU CV/LASSO/DML tests, then a short bench per setting under a kernel trace
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local n=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$n.log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] failed rc=$rc"; tail -30 "$OUT/$n.log"; exit $rc; fi
  echo "[$n] ok: $(tail -1 "$OUT/$n.log" | cut -c1-200)"; }
step tests 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_panel_selection.py tests/test_gpu_multirank.py -x -q --timeout 200 --timeout-method thread -k "cv or lasso or dml or enet or bench or exact"
R=$PWD
cd /tmp
for v in 1 4 2 8 4 1; do
  ATE_CVL_PARTS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_$v -- python3 $R/bench.py --steps 20 --parity 0 --also-rct 0 --repeats 1 --inflight 1 > $R/$OUT/bench_$v.log 2>&1 || exit $?
  echo "parts $v: $(grep -o '"ms_per_step": [0-9.]*' $R/$OUT/bench_$v.log) $(grep -o '"ate_hex": "[^"]*"' $R/$OUT/bench_$v.log | head -1) $(grep -o '"se_hex": "[^"]*"' $R/$OUT/bench_$v.log | head -1)"
done
