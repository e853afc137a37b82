#!/bin/bash
# A/B the bench step on one box: the in-tree library vs _lib/libatehip_base.so (built with
# tools/build_variant.py), alternating, N rounds: the CV-LASSO stage alone, then the step
# (ms/step, ATE, SE so bit-identity is visible). Usage: bash tools/ab_bench.sh [rounds]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
BASE=$R/ate_replication_causalml_amd/_lib/libatehip_base.so
ms() { python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step'], 3), 'single', round(d['single_fit_ms'], 3), repr(d['ate']), repr(d['se']))" "$1"; }
for i in $(seq ${1:-2}); do
  timeout -k 10 200 python $R/tools/enet_only.py 10 | sed 's/^/new  /' || exit 1
  ATE_HIP_LIB=$BASE timeout -k 10 200 python $R/tools/enet_only.py 10 | sed 's/^/base /' || exit 1
  timeout -k 10 300 python $R/bench.py --steps 10 --warmup 3 | ms new || exit 1
  ATE_HIP_LIB=$BASE timeout -k 10 300 python $R/bench.py --steps 10 --warmup 3 | ms base || exit 1
done
