#!/bin/bash
# A/B the bench step on one box: the in-tree library vs _lib/libatehip_base.so (a build of
# the previous revision), alternating, N rounds: the CV-LASSO stage alone, then the step. Usage: bash tools/ab_bench.sh [rounds]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
BASE=$R/ate_replication_causalml_amd/_lib/libatehip_base.so
ms() { python -c "import json,sys; print(sys.argv[1], round(json.loads(sys.stdin.read())['ms_per_step'], 3))" "$1"; }
for i in $(seq ${1:-2}); do
  timeout -k 10 200 python $R/tools/enet_only.py 10 | sed 's/^/new  /' || exit 1
  ATE_HIP_LIB=$BASE timeout -k 10 200 python $R/tools/enet_only.py 10 | sed 's/^/base /' || exit 1
  timeout -k 10 300 python $R/bench.py --steps 10 --warmup 3 | ms new || exit 1
  ATE_HIP_LIB=$BASE timeout -k 10 300 python $R/bench.py --steps 10 --warmup 3 | ms base || exit 1
done
