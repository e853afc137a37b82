#!/bin/bash
# Round-6: fused root pass (interleaved (g, h) pairs, computed rows for a fold's complement):
# GBDT GPU tests, then the config-5 shard (10 trees per model): fused unroll 4 (in tree),
# fused unroll 8 (libatehip_u8), and one fit after the other (ATE_GBDT_FUSED_ROOT=0)
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
L=$PWD/ate_replication_causalml_amd/_lib
step() { local n=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$n.log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] failed rc=$rc"; tail -30 "$OUT/$n.log"; exit $rc; fi
  echo "[$n] ok: $(tail -1 "$OUT/$n.log" | grep -o '"seconds": [0-9.]*, ' ) $(tail -1 "$OUT/$n.log" | grep -o '"ate": [0-9.]*') $(tail -1 "$OUT/$n.log" | grep -o 'passed.*')"; }
step tests 400 python -u -m pytest tests/test_gbdt_gpu.py -x -q --timeout 200 --timeout-method thread
for i in 1 2; do
  step u4_$i 300 python -u tools/cfg5.py --rows 1e8 --cols 2000 --trees 10 --shard 0/8
  ATE_HIP_LIB=$L/libatehip_u8.so step u8_$i 300 python -u tools/cfg5.py --rows 1e8 --cols 2000 --trees 10 --shard 0/8
  ATE_GBDT_FUSED_ROOT=0 step serial_$i 300 python -u tools/cfg5.py --rows 1e8 --cols 2000 --trees 10 --shard 0/8
done
R=$PWD
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -- python3 $R/tools/cfg5.py --rows 1e8 --cols 2000 --trees 10 --shard 0/8 > $R/$OUT/prof.log 2>&1 && echo profiled
