#!/bin/bash
# PMC counter passes over one config-3 forest (tools/forest_level_probe.py: 13 trees of the
# per-GPU shard's fold-0 propensity forest, N=2e6 panel -> 1.6e6 training rows) on the level
# engine (csrc/forest_level.hip) and the per-tree kernel (csrc/forest.hip forest_grow_kernel).
# One counter set per rocprofv3 run, kernel-trace only; stops at the first fault-class exit.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_forest
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "TCC_HIT_sum TCC_MISS_sum" \
           "FETCH_SIZE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  for eng in level tree; do
    N=2e6 ENGINES=$eng timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $set --output-format csv \
        -d $OUT/${eng}_set$i -- python3 $R/tools/forest_level_probe.py > $OUT/${eng}_set$i.log 2>&1
    rc=$?
    echo "$eng set$i ($set) rc=$rc"
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
python3 $R/tools/pmc_forest_summary.py $OUT | tee $OUT/summary.txt
exit 0
