#!/bin/bash
# PMC passes over the CV-LASSO stage alone (tools/enet_only.py, N=1e7 p=500 bench Grams):
# L2 hit/miss and fetch size of the path kernel; one counter set per run.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_enet
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/set$i -- \
      python3 $R/tools/enet_only.py 3 > $OUT/set$i.log 2>&1
  rc=$?
  echo "set$i ($set) rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
python3 $R/tools/pmc_summary.py $OUT enet_path
exit 0
