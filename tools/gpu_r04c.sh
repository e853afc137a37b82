#!/bin/bash
# config 3 after the packed-C05 refactor: forest/multirank GPU tests, then the per-GPU
# shard of the named config (N=1e7, p=500, 100 trees/forest, rank 0 of 8)
set -o pipefail
OUT=gpurun_out/r04c; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_forest_gpu.py tests/test_gpu_multirank.py -k "cfg3 or crossfit or panel" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/tests.log | head; exit $rc; }
timeout -k 10 240 python -u tools/cfg3.py --rows 10000000 --cols 500 --trees 100 --shard 0/8 > $OUT/cfg3_shard.log 2>&1 || { echo cfg3 failed; tail -5 $OUT/cfg3_shard.log; exit 1; }
tail -1 $OUT/cfg3_shard.log
