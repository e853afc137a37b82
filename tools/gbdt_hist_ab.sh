#!/bin/bash
# Level-0 histogram kernel time, in-tree library vs a variant (_lib/libatehip_$1.so): kernel
# trace of a 2-tree config-5 shard run; the hist launches of level 0 are every 6th call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/gbdt_ab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in new "$@"; do
  if [ $v = new ]; then unset ATE_HIP_LIB; else export ATE_HIP_LIB=$R/ate_replication_causalml_amd/_lib/libatehip_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$v -o kt -- \
      python3 $R/tools/cfg5.py --rows 100000000 --cols 2000 --trees 2 --shard 0/8 > $OUT/$v.log 2>&1 || { echo "$v failed"; tail -3 $OUT/$v.log; exit 1; }
  python3 - "$OUT/$v" "$v" <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gbdt_hist_kernel" in r["Kernel_Name"]:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
rows.sort()
d = [x[1] / 1e6 for x in rows]
lv0 = d[0::6]
print(sys.argv[2], "hist calls", len(d), "total ms", round(sum(d), 1), "level-0 mean ms", round(sum(lv0) / len(lv0), 2),
      "level-1..5 mean ms", [round(sum(d[k::6]) / len(d[k::6]), 2) for k in range(1, 6)])
PY
done
