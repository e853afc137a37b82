#!/bin/bash
# Round-6: how far a fold path may run ahead of its source (ENET_FOLD_LEAD 2 in tree vs
# 3/4/6 variant libraries): enet GPU tests on each library, then the CV-LASSO stage of
# the bench (tools/enet_only.py) alternated over the libraries, tutorial and RCT designs
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
L=$PWD/ate_replication_causalml_amd/_lib
step() { local n=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$n.log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] failed rc=$rc"; tail -30 "$OUT/$n.log"; exit $rc; fi
  echo "[$n] ok: $(tail -1 "$OUT/$n.log" | cut -c1-200)"; }
sel() { if [ "$1" = lead2 ]; then unset ATE_HIP_LIB; else export ATE_HIP_LIB=$L/libatehip_$1.so; fi; }
for v in lead2 lead4; do
  sel $v; step tests_$v 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "cv or lasso or enet or repeated"
done
for dgp in tutorial rct; do
  export ATE_DGP=$dgp
  for r in 1 2; do
    for v in lead2 lead3 lead4 lead6; do
      sel $v; step ${dgp}_${v}_$r 200 python -u tools/enet_only.py 30
    done
  done
done
