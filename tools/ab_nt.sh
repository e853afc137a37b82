#!/bin/bash
# Gram alone and the bench step: in-tree library vs libatehip_nt.so (nt panel stream).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
V=$R/ate_replication_causalml_amd/_lib/libatehip_nt.so
ms() { python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step'], 3), 'single', round(d['single_fit_ms'], 3), repr(d['ate']))" "$1"; }
for i in 1 2; do
  timeout -k 10 200 python $R/tools/gram_only.py 1e7 | sed 's/^/base /' || exit 1
  ATE_HIP_LIB=$V timeout -k 10 200 python $R/tools/gram_only.py 1e7 | sed 's/^/nt   /' || exit 1
  timeout -k 10 300 python $R/bench.py --steps 20 --warmup 3 | ms base || exit 1
  ATE_HIP_LIB=$V timeout -k 10 300 python $R/bench.py --steps 20 --warmup 3 | ms nt || exit 1
done
