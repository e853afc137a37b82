#!/bin/bash
# Multi-rank rehearsal on ONE GPU: W ranks share the card, collectives over gloo (host-
# staged), everything else as in the RCCL run (three fits in flight, staggered streams,
# sharded path solves). Compares rank 0's ATE/SE with one process holding all the rows.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
ROWS=${ROWS:-2000000}
for W in ${WORLDS:-2 3}; do
  ATE_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W \
    --master-addr 127.0.0.1 --master-port $((29600 + W)) $R/bench.py --gpus $W --rows $ROWS --steps 5 --warmup 2 --parity 0 \
    > $R/gpurun_out/rehearse_$W.log 2>&1 || { echo "world $W failed"; tail -20 $R/gpurun_out/rehearse_$W.log; exit 1; }
  timeout -k 10 300 python $R/bench.py --rows $((ROWS * W)) --steps 2 --warmup 1 --parity 0 > $R/gpurun_out/rehearse_1x$W.log 2>&1 || exit 1
  python - $R/gpurun_out/rehearse_$W.log $R/gpurun_out/rehearse_1x$W.log $W <<'PY'
import json, sys
a = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
b = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(f"world {sys.argv[3]}: ranks ate={a['ate']!r} se={a['se']!r} | one process ate={b['ate']!r} se={b['se']!r} | "
      f"diff {abs(a['ate'] - b['ate']):.2e} {abs(a['se'] - b['se']):.2e} | hipgraph {a['hipgraph']} inflight {a.get('throughput_inflight')}")
PY
done
