#!/bin/bash
# Round-6: GBDT level-histogram workgroups of 16 features (GBDT_FB=16, libatehip_fb16) vs 32
# (in tree), config-5 shard, 10 trees, fused root in both
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
L=$PWD/ate_replication_causalml_amd/_lib
step() { local n=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$n.log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] failed rc=$rc"; tail -30 "$OUT/$n.log"; exit $rc; fi
  echo "[$n] ok: $(tail -1 "$OUT/$n.log" | grep -o '"seconds": [0-9.]*, ' ) $(tail -1 "$OUT/$n.log" | grep -o '"ate": [0-9.]*')"; }
step warm 300 python -u tools/cfg5.py --rows 1e8 --cols 2000 --trees 2 --shard 0/8
for i in 1 2; do
  step fb32_$i 300 python -u tools/cfg5.py --rows 1e8 --cols 2000 --trees 10 --shard 0/8
  ATE_HIP_LIB=$L/libatehip_fb16.so step fb16_$i 300 python -u tools/cfg5.py --rows 1e8 --cols 2000 --trees 10 --shard 0/8
done
