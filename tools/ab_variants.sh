#!/bin/bash
# CV-LASSO stage time and bench ATE/SE for the in-tree library and each _lib/libatehip_<v>.so
# named on the command line. Usage: bash tools/ab_variants.sh base all half
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
ms() { python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step'], 3), 'single', round(d['single_fit_ms'], 3), repr(d['ate']), repr(d['se']))" "$1"; }
timeout -k 10 200 python $R/tools/enet_only.py 10 | sed 's/^/new  /' || exit 1
for v in "$@"; do
  ATE_HIP_LIB=$R/ate_replication_causalml_amd/_lib/libatehip_$v.so timeout -k 10 200 python $R/tools/enet_only.py 10 | sed "s/^/$v /" || exit 1
done
timeout -k 10 300 python $R/bench.py --steps 10 --warmup 3 | ms new || exit 1
for v in "$@"; do
  ATE_HIP_LIB=$R/ate_replication_causalml_amd/_lib/libatehip_$v.so timeout -k 10 300 python $R/bench.py --steps 10 --warmup 3 | ms $v || exit 1
done
