#!/bin/bash
# Round-6: CV-loss kernel with 4 lambdas per workgroup (libatehip_cvl4) vs 8 (in tree):
# GPU enet/lasso tests, then kernel stats of a short bench run per library
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
L=$PWD/ate_replication_causalml_amd/_lib
step() { local n=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$n.log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] failed rc=$rc"; tail -30 "$OUT/$n.log"; exit $rc; fi
  echo "[$n] ok: $(tail -1 "$OUT/$n.log" | cut -c1-200)"; }
step tests 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "cv or lasso or dml or enet"
R=$PWD
cd /tmp
for v in new cvl4 new cvl4; do
  if [ $v = cvl4 ]; then export ATE_HIP_LIB=$L/libatehip_cvl4.so; else unset ATE_HIP_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_$v -- python3 $R/bench.py --steps 20 --parity 0 --also-rct 0 --repeats 1 --inflight 1 > $R/$OUT/bench_$v.log 2>&1 || exit $?
  echo "$v: $(grep -o '"ms_per_step": [0-9.]*' $R/$OUT/bench_$v.log) $(grep -o '"ate_hex": "[^"]*"' $R/$OUT/bench_$v.log | head -1)"
done
