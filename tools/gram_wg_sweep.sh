#!/bin/bash
# Bench step at several Gram workgroup targets (equal-chunk planner); pass targets as args.
mkdir -p gpurun_out
for wg in "$@"; do
  echo "bench wg=$wg $(ATE_GRAM_PAIR_WG=$wg timeout -k 10 200 python bench.py 2>/dev/null | tail -1 | cut -c150-300)" || exit 1
done
