#!/bin/bash
# Round-6 A/B: balanced diagonal-pair waves (GRAM_BAL=1, in tree) vs 32/36 (libatehip_nobal)
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
L=$PWD/ate_replication_causalml_amd/_lib
step() { local n=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$n.log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] failed rc=$rc"; tail -30 "$OUT/$n.log"; exit $rc; fi
  echo "[$n] ok: $(tail -2 "$OUT/$n.log" | tr '\n' ' ' | cut -c1-300)"; }
step tests 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "gram or dml"
for v in new nobal new nobal; do
  lib=$L/libatehip_$v.so; [ $v = new ] && lib=$L/libatehip.so
  ATE_HIP_LIB=$lib ATE_GRAM_STAGE=tiles step gram_$v 200 python -u tools/gram_only.py 1e7 pair pair
done
for v in new nobal new nobal; do
  lib=$L/libatehip_$v.so; [ $v = new ] && lib=$L/libatehip.so
  ATE_HIP_LIB=$lib step single_$v 300 python -u tools/single_ab.py pair 3 20
done
