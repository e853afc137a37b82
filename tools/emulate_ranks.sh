#!/bin/bash
# Rank 0's share of the world-W bench step on one GPU (ATE_BENCH_EMULATE_WORLD: its row
# shard of W x 1e7 rows, its outer folds' path solves, no-op collectives): projects the
# per-rank step time of the multi-GPU runs without the RCCL cost.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for w in ${WORLDS:-1 2 4 8}; do
  ATE_BENCH_EMULATE_WORLD=$w timeout -k 10 300 python $R/bench.py --steps 20 --warmup 3 $BARGS > $R/gpurun_out/emu_$w.log 2>&1 || { echo "fail $w"; tail -5 $R/gpurun_out/emu_$w.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); print('world', sys.argv[1], 'ms/step', round(d['ms_per_step'],3), 'single', round(d['single_fit_ms'],3))" $w $R/gpurun_out/emu_$w.log | tee -a $R/gpurun_out/emulate.log
done
