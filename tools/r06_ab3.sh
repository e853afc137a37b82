#!/bin/bash
# Round-6 A/B 3: gram tests; tile kernel alone: pair / tri (3 type-0 stages, in tree) /
# tri with 2 type-0 stages (libatehip_s2.so); single-call A/B tri vs pair on one panel.
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local n=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$n.log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] failed rc=$rc"; tail -30 "$OUT/$n.log"; exit $rc; fi
  echo "[$n] ok: $(tail -2 "$OUT/$n.log" | cut -c1-300)"; }
step tests 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "gram"
ATE_GRAM_STAGE=tiles step gram_tiles 200 python -u tools/gram_only.py 1e7 pair tri pair tri
ATE_GRAM_STAGE=tiles ATE_HIP_LIB=$PWD/ate_replication_causalml_amd/_lib/libatehip_s2.so step gram_tiles_s2 200 python -u tools/gram_only.py 1e7 tri tri
step single_ab 300 python -u tools/single_ab.py tri,pair 4 20
