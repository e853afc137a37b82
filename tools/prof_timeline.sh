#!/bin/bash
# Kernel trace of a bench run (extra args in BARGS, env passed through) + tools/timeline.py
# listing of its overlapped part -> gpurun_out/prof_tl/timeline.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/prof_tl
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_tl -o tl \
  -- python3 $R/bench.py --steps ${STEPS:-8} --warmup 2 $BARGS > $R/gpurun_out/prof_tl/bench.log 2>&1 || { echo prof failed; tail -5 $R/gpurun_out/prof_tl/bench.log; exit 1; }
python3 -c "import sys; sys.path.insert(0, '$R/tools'); import timeline; timeline.overlapped(sys.argv[1], 400)" $(find $R/gpurun_out/prof_tl -name "*kernel_trace.csv") > $R/gpurun_out/prof_tl/timeline.txt
tail -1 $R/gpurun_out/prof_tl/bench.log | cut -c1-300
