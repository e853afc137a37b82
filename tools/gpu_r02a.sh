#!/bin/bash
# Round-2 check: segmented-graph tests with real RCCL, GPU suite, bench (1 rank), 2-rank gloo rehearsal.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_segmented.py tests/test_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/seg_tests.log 2>&1 || { echo "seg tests failed"; tail -40 gpurun_out/seg_tests.log; exit 1; }
tail -3 gpurun_out/seg_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
ATE_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --rows 2e6 > gpurun_out/bench2.log 2>&1 || { echo bench2 failed; tail -30 gpurun_out/bench2.log; exit 1; }
grep metric gpurun_out/bench2.log
echo done
