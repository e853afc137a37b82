#!/bin/bash
# PMC counter passes over a short config-5 GBDT run (one counter set per rocprofv3 run,
# kernel-trace only; stops at the first fault-class exit status).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_gbdt
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/avail.txt 2>&1
i=0
for set in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES" \
           "SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/set$i -- \
      python3 $R/tools/bench_configs.py --configs 5 --trees5 2 --n5 1000000 > $OUT/set$i.log 2>&1
  rc=$?
  echo "set$i ($set) rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
exit 0
