#!/bin/bash
# Forest growth time per waves-per-tree setting (ATE_FOREST_NW; 0 = the automatic choice in
# csrc/forest.hip ate_forest_fit) at n = 1e6 (64 / 300 trees) and the tutorial shape.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for nw in ${NWS:-0 4 8 16}; do
  ATE_FOREST_NW=$nw timeout -k 10 300 python $R/tools/forest_grow_time.py 2>&1 | grep -v amdgpu.ids | sed "s/^/nw=$nw /" || exit 1
done
