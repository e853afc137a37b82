#!/bin/bash
# Round-6: in-flight Gram workgroup count (ATE_GRAM_PAIR_WG) with the byte columns
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2; do
  for wg in 1024 1536 2048 2560 3072; do
    ATE_GRAM_PAIR_WG=$wg timeout -k 10 200 python -u bench.py --parity 0 --also-rct 0 --repeats 1 > $OUT/wg${wg}_$i.log 2>&1 || exit $?
    echo "wg $wg: $(grep -o '"throughput_inflight": {"inflight": 3, "ms_per_fit": [0-9.]*' $OUT/wg${wg}_$i.log | grep -o '[0-9.]*$') single $(grep -o '"ms_per_step": [0-9.]*' $OUT/wg${wg}_$i.log | head -1)"
  done
done
