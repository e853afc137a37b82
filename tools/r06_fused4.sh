#!/bin/bash
# Round-6: level-kernel chunk length (ATE_GBDT_HIST_ROWS) with the fused root at 65536 rows,
# config-5 shard, 10 trees
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local n=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$n.log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] failed rc=$rc"; tail -30 "$OUT/$n.log"; exit $rc; fi
  echo "[$n] ok: $(tail -1 "$OUT/$n.log" | grep -o '"seconds": [0-9.]*, ' ) $(tail -1 "$OUT/$n.log" | grep -o '"ate": [0-9.]*')"; }
for i in 1 2; do
  for r in ${ROWS:-65536 131072 262144}; do
    ATE_GBDT_HIST_ROWS=$r step r${r}_$i 300 python -u tools/cfg5.py --rows 1e8 --cols 2000 --trees 10 --shard 0/8
  done
done
