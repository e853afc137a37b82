#!/bin/bash
# Gram alone (tools/gram_only.py, N=1e7 bench panel) for the in-tree library and each
# _lib/libatehip_<v>.so named on the command line, alternating twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for i in 1 2; do
  timeout -k 10 200 python $R/tools/gram_only.py 1e7 | sed 's/^/base /' || exit 1
  for v in "$@"; do
    ATE_HIP_LIB=$R/ate_replication_causalml_amd/_lib/libatehip_$v.so timeout -k 10 200 python $R/tools/gram_only.py 1e7 | sed "s/^/$v /" || exit 1
  done
done
