#!/bin/bash
# Level-0 histogram kernel time per ablation mode (ATE_GBDT_HIST_MODE: 1 no LDS atomics,
# 2 no bins gather, 4 no slab store, 8 G atomics only). Level 0 histograms every training
# row whatever the earlier trees were, so its time is a valid breakdown (deeper levels are
# not: a corrupted histogram changes the splits and the later levels' work).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/gbdt_modes_l0
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for m in ${MODES:-0 1 2 4 8}; do
  ATE_GBDT_HIST_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/m$m -o kt -- \
      python3 $R/tools/cfg5.py --rows 100000000 --cols 2000 --trees 1 --shard 0/8 > $OUT/m$m.log 2>&1 || { echo "mode $m failed"; tail -3 $OUT/m$m.log; exit 1; }
  python3 - "$OUT/m$m" "$m" <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gbdt_hist_kernel" in r["Kernel_Name"]:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
rows.sort()
d = [x[1] / 1e6 for x in rows]
lv0 = d[0::6]
print("mode", sys.argv[2], "level-0 hist ms", round(sum(lv0) / len(lv0), 2), "of", len(lv0), "fits")
PY
done
