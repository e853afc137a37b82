#!/bin/bash
# Round-6: config-5 per-GPU shard, 100 trees per model (fused root, 64k-row chunks), plus
# the GBDT GPU tests
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local n=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$n.log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] failed rc=$rc"; tail -30 "$OUT/$n.log"; exit $rc; fi
  echo "[$n] ok: $(tail -1 "$OUT/$n.log" | grep -o '"seconds": [0-9.]*, ' ) $(tail -1 "$OUT/$n.log" | grep -o '"ate": [0-9.]*') $(tail -1 "$OUT/$n.log" | grep -o '[0-9]* passed.*')"; }
step tests 400 python -u -m pytest tests/test_gbdt_gpu.py -x -q --timeout 200 --timeout-method thread
step fused 400 python -u tools/cfg5.py --rows 1e8 --cols 2000 --trees 100 --shard 0/8
step fused2 400 python -u tools/cfg5.py --rows 1e8 --cols 2000 --trees 100 --shard 0/8
