#!/bin/bash
# PMC counter passes over the standalone bf16 Gram (tools/gram_only.py, N=1e7, p=500);
# one counter set per rocprofv3 run, kernel-trace only; stops at a fault-class exit.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_gram
V=${1:-}            # optional Gram variant name (gram_only.py), default: the library default
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "TCC_HIT_sum TCC_MISS_sum" \
           "FETCH_SIZE" \
           "TA_BUSY_avr TD_BUSY_avr GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/v${V:-default}/set$i -- \
      python3 $R/tools/gram_only.py 1e7 $V > $OUT/v${V:-default}.set$i.log 2>&1
  rc=$?
  echo "set$i ($set) rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
exit 0
