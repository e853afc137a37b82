#!/bin/bash
# kernel trace of the single-call A/B (tools/single_ab.py): per-kernel time, tri vs pair
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
for v in tri pair; do
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$ROOT/$OUT/prof_$v" -o k -- python3 "$ROOT/tools/single_ab.py" $v 2 10 \
      > "$ROOT/$OUT/prof_$v.log" 2>&1 ) || { echo "[prof_$v] failed"; tail -20 "$OUT/prof_$v.log"; exit 1; }
  tail -1 "$OUT/prof_$v.log"
  f=$(find "$OUT/prof_$v" -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]:
    print(f"  {r['Name'][:60]:60s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:9.1f}")
PY
done
