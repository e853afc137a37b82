#!/bin/bash
# A/B kernel statistics of bench.py per library: tools/prof_ab.sh OUT A,B,..
# ("new" = the in-tree libatehip.so, NAME = _lib/libatehip_NAME.so); rocprofv3 kernel
# trace + stats of a short bench run on both panels, summaries under OUT/prof_NAME/
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$1
mkdir -p "$OUT"
IFS=, read -ra libs <<< "$2"
for nm in "${libs[@]}"; do
  lib=$ROOT/ate_replication_causalml_amd/_lib/libatehip_$nm.so
  [ "$nm" = new ] && lib=$ROOT/ate_replication_causalml_amd/_lib/libatehip.so
  ( cd /tmp && export TMPDIR=/tmp ATE_HIP_LIB=$lib && timeout -k 10 300 rocprofv3 --kernel-trace \
      --stats --output-format csv -d "$OUT/prof_$nm" -o bench -- python3 "$ROOT/bench.py" \
      --steps 5 --warmup 1 --parity 0 > "$OUT/prof_$nm.log" 2>&1 ) || { echo "[$nm] failed"; exit 1; }
  echo "[$nm] ok"
done
