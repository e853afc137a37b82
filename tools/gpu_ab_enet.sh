#!/bin/bash
# A/B of CV-path-kernel builds: enet tests, then the CV-LASSO stage alone
# (tools/enet_only.py) for each named library, alternating, then the bench.
#   bash tools/gpu_ab_enet.sh OUTDIR name1 name2 ...   (libatehip_<name>.so; "new" = in-tree)
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py tests/test_gpu_determinism.py -k "enet or lasso or dml or belloni or determinism" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for nm in "$@"; do
    lib=ate_replication_causalml_amd/_lib/libatehip_$nm.so
    [ "$nm" = new ] && lib=ate_replication_causalml_amd/_lib/libatehip.so
    ATE_HIP_LIB=$PWD/$lib timeout -k 10 120 python tools/enet_only.py 15 > $OUT/enet_$nm.$rep.log 2>&1 || { echo "enet_only $nm failed"; tail -5 $OUT/enet_$nm.$rep.log; exit 1; }
    echo "$nm $(tail -1 $OUT/enet_$nm.$rep.log)"
  done
done
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { echo bench failed; tail -20 $OUT/bench.log; exit 1; }
python - $OUT/bench.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("bench", round(d["ms_per_step"], 3), "single", round(d["single_fit_ms"], 3), d["ate_hex"], d["se_hex"], d["parity"]["abs_diff_ate"])
PY
