#!/bin/bash
# Round-6 PMC passes over the standalone paired-tile Gram (tools/gram_only.py, N=1e7,
# p=500): the all-bf16 read (pair16, the default path) and the one-byte binary columns
# (pair). One counter set per rocprofv3 run, kernel-trace only; stops at a fault-class exit.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06_pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for V in pair16 pair; do
  i=0
  for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
             "TCC_HIT_sum TCC_MISS_sum" \
             "FETCH_SIZE" \
             "TA_BUSY_avr TD_BUSY_avr GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/$V/set$i -- \
        python3 $R/tools/gram_only.py 1e7 $V $V $V $V > $OUT/$V.set$i.log 2>&1
    rc=$?
    echo "$V set$i ($set) rc=$rc"
    case $rc in 124|134|137|139) exit $rc;; esac
  done
  python3 $R/tools/pmc_summary.py $OUT/$V gram_bf16_pair > $OUT/${V}_summary.txt
done
exit 0
