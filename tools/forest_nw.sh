#!/bin/bash
# Waves per tree (ATE_FOREST_NW) A/B: forest GPU tests (bit-identity with the host engine)
# and large-N fit time for each setting.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for nw in ${NWS:-4 8 16}; do
  ATE_FOREST_NW=$nw timeout -k 10 400 python -u -m pytest $R/tests/test_forest_gpu.py -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/fnw_test_$nw.log 2>&1 || { echo "tests failed nw=$nw"; tail -20 $R/gpurun_out/fnw_test_$nw.log; exit 1; }
  echo "nw=$nw tests: $(tail -1 $R/gpurun_out/fnw_test_$nw.log)"
  ATE_FOREST_NW=$nw timeout -k 10 400 python $R/tools/rf_scale_probe.py 2>&1 | grep -v amdgpu.ids | sed "s/^/nw=$nw /" || exit 1
done
