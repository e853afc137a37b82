#!/bin/bash
# Histogram-kernel ablation on config 5 (run on the GPU box from the repo root):
#   ATE_GBDT_HIST_MODE bits: 1 = skip the LDS atomics, 2 = synthetic bins (no bin loads),
#   4 = skip the slab store;  ATE_GBDT_HIST_TARGET = histogram workgroups per level.
# usage: tools/gbdt_ablation.sh "MODE TARGET" ...   (default: "0 512" "1 512" "3 512")
# then:  python tools/kstats.py gpurun_out/abl_<MODE>_<TARGET> --cycle hist_kernel=6
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
[ $# -eq 0 ] && set -- "0 512" "1 512" "3 512"
for cfg in "$@"; do
  set -- $cfg
  ATE_GBDT_HIST_MODE=$1 ATE_GBDT_HIST_TARGET=$2 timeout -k 10 200 rocprofv3 --kernel-trace \
      --output-format csv -d $R/gpurun_out/abl_$1_$2 -- \
      python3 $R/tools/bench_configs.py --configs 5 --trees5 3 > $R/gpurun_out/abl_$1_$2.log 2>&1
  rc=$?; echo "cfg $cfg rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
