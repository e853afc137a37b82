#!/bin/bash
# Round-6: config-3 per-GPU shard (tutorial panel), timing + kernel stats
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
R=$PWD
timeout -k 10 300 python -u tools/cfg3.py --rows 1e7 --cols 500 --trees 100 --shard 0/8 > $OUT/cfg3.log 2>&1 || exit $?
echo "cfg3: $(tail -1 $OUT/cfg3.log | grep -o '"seconds": [0-9.]*')"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -- python3 $R/tools/cfg3.py --rows 1e7 --cols 500 --trees 100 --shard 0/8 > $R/$OUT/cfg3_prof.log 2>&1 || exit $?
echo profiled
