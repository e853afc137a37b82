#!/bin/bash
# Round-6: where the byte path's time goes -- the tile kernel with the byte columns as bf16
# (pair16), as bytes (pair), and as bytes without the v_perm conversion (noperm build,
# timing only: wrong values)
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
L=$PWD/ate_replication_causalml_amd/_lib
step() { local n=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$n.log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] failed rc=$rc"; tail -30 "$OUT/$n.log"; exit $rc; fi
  echo "[$n] ok: $(grep kernel "$OUT/$n.log" | tr '\n' ' ' | cut -c1-400)"; }
ATE_GRAM_STAGE=tiles step gram_new 200 python -u tools/gram_only.py 1e7 pair16 pair pair16 pair
ATE_GRAM_STAGE=tiles ATE_HIP_LIB=$L/libatehip_noperm.so step gram_noperm 200 python -u tools/gram_only.py 1e7 pair16 pair pair16 pair
