#!/bin/bash
# Round-6: one-byte columns in the paired-tile Gram -- GPU tests, tile kernel alone and the
# single call, bytes (pair) vs the same panel read as bf16 (pair16), then bench.py.
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local n=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$n.log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] failed rc=$rc"; tail -30 "$OUT/$n.log"; exit $rc; fi
  echo "[$n] ok: $(tail -2 "$OUT/$n.log" | tr '\n' ' ' | cut -c1-400)"; }
step tests 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_panel_selection.py -x -q --timeout 200 --timeout-method thread -k "gram or byte or dml or selection or repeated"
ATE_GRAM_STAGE=tiles step gram_tiles 200 python -u tools/gram_only.py 1e7 pair pair16 pair pair16
step single_ab 400 python -u tools/single_ab.py pair,pair16 4 20
step bench 400 python -u bench.py
