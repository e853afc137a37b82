#!/bin/bash
# PMC passes over the config-5 GBDT histogram kernel (one tree per nuisance model of the
# per-GPU shard, N=1.25e7 x p=2000): one counter set per rocprofv3 run.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_gbdt5
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/set$i -- \
      python3 $R/tools/cfg5.py --rows 100000000 --cols 2000 --trees 1 --shard 0/8 > $OUT/set$i.log 2>&1
  rc=$?
  echo "set$i ($set) rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
python3 - "$OUT" <<'PY'
import collections, csv, glob, sys
out = sys.argv[1]
per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/**/*_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gbdt_hist_kernel" not in r["Kernel_Name"]:
            continue
        per[r["Counter_Name"]][int(r["Dispatch_Id"])].append(float(r["Counter_Value"]))
for c, d in sorted(per.items()):
    ids = sorted(d)
    vals = [sum(d[i]) for i in ids]
    print(c, "dispatches", len(vals), "first (level 0):", f"{vals[0]:.4g}", "all:", " ".join(f"{v:.3g}" for v in vals[:6]))
PY
