#!/bin/bash
# Round-6: the level engine's mid-node accumulate with the next step's row indices loaded
# behind this step's gathers (LV_RK_PF) and/or 16 rows per lane in flight (LV_RK_U), as
# variant libraries against the in-tree build: forest GPU tests on the prefetch build,
# then the config-3 per-GPU shard alternated over the libraries
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
L=$PWD/ate_replication_causalml_amd/_lib
step() { local n=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$n.log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] failed rc=$rc"; tail -30 "$OUT/$n.log"; exit $rc; fi
  echo "[$n] ok: $(tail -1 "$OUT/$n.log" | cut -c1-200)"; }
sel() { if [ "$1" = base ]; then unset ATE_HIP_LIB; else export ATE_HIP_LIB=$L/libatehip_$1.so; fi; }
sel pf16; step tests_pf16 400 python -u -m pytest tests/test_forest_gpu.py -x -q --timeout 200 --timeout-method thread
for v in base pf pf16 u16 pf4 base pf pf16; do
  sel $v
  timeout -k 10 300 python -u tools/cfg3.py --rows 1e7 --cols 500 --trees 100 --shard 0/8 > $OUT/cfg3_$v.log 2>&1 || exit $?
  echo "$v: $(tail -1 $OUT/cfg3_$v.log | grep -o '"seconds": [0-9.]*') $(tail -1 $OUT/cfg3_$v.log | grep -o '"ate_hex": "[^"]*"')"
done
