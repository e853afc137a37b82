#!/bin/bash
# kernel summary + trace of the config-3 per-GPU shard (N=1e7 x 500, 13 of 100 trees of
# each of the 15 forests) at the package's default forest concurrency
set -o pipefail
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_configs.py --configs 3 --panel3 --n3 10000000 --p3 500 --shard3 0/8 --trees3 100 > gpurun_out/cfg3_plain.log 2>&1 || { echo cfg3 failed; tail -5 gpurun_out/cfg3_plain.log; exit 1; }
tail -1 gpurun_out/cfg3_plain.log | cut -c 1-400
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_cfg3" -o cfg3 \
  -- python3 "$ROOT/tools/bench_configs.py" --configs 3 --panel3 --n3 10000000 --p3 500 --shard3 0/8 --trees3 100 > "$ROOT/gpurun_out/prof_cfg3.log" 2>&1 || { echo prof failed; tail -5 "$ROOT/gpurun_out/prof_cfg3.log"; exit 1; }
f=$(find $ROOT/gpurun_out/prof_cfg3 -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(r["Name"][:70], r["Calls"], round(float(r["TotalDurationNs"]) / 1e6, 1), r["Percentage"][:5])
PY
