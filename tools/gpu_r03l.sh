#!/bin/bash
# Round-3 re-entry check: gpu tests, smoke, bench + kernel profile, then the per-level
# config-5 histogram kernel times of the current (32k-row chunk) build.
set -o pipefail
bash tools/gpu_check.sh || exit 1
bash tools/gbdt_hist_ab.sh > gpurun_out/gbdt_levels.log 2>&1 || { tail -5 gpurun_out/gbdt_levels.log; exit 1; }
cat gpurun_out/gbdt_levels.log
