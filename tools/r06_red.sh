#!/bin/bash
# Round-6: the Gram's fixed-order slab reduce with 16 / 32 chunk loads in flight per
# thread (GRAM_RED_U; 8 in tree), same summation order: Gram GPU tests on the U=32 build,
# then kernel stats of a short single-call bench per library, alternated
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
L=$PWD/ate_replication_causalml_amd/_lib
step() { local n=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$n.log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] failed rc=$rc"; tail -30 "$OUT/$n.log"; exit $rc; fi
  echo "[$n] ok: $(tail -1 "$OUT/$n.log" | cut -c1-200)"; }
export ATE_HIP_LIB=$L/libatehip_red32.so
step tests 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "gram or dml or byte"
R=$PWD
cd /tmp
for v in base red16 red32 base red16 red32; do
  if [ $v = base ]; then unset ATE_HIP_LIB; else export ATE_HIP_LIB=$L/libatehip_$v.so; fi
  D=/tmp/prof_$v; rm -rf $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -- python3 $R/bench.py --steps 20 --parity 0 --also-rct 0 --repeats 1 --inflight 0 > $R/$OUT/bench_$v.log 2>&1 || exit $?
  f=$(find $D -name '*kernel_stats.csv' | head -1)
  echo "$v: $(grep -o '"ms_per_step": [0-9.]*' $R/$OUT/bench_$v.log) $(grep -o '"ate_hex": "[^"]*"' $R/$OUT/bench_$v.log | head -1) $(python3 -c "import csv,sys; [print(r['Name'].split('(')[0][:28], r['Calls'], r['AverageNs'], end='; ') for r in csv.DictReader(open(sys.argv[1])) if 'reduce' in r['Name']]" $f)"
done
