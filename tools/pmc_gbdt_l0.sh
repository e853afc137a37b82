#!/bin/bash
# PMC passes over the config-5 histogram kernel (1 tree per model): per-level values of
# instruction mix, VMEM / LDS waits and TA / TCP stalls. One counter set per run.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_gbdt_l0
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" \
           "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/set$i -- \
      python3 $R/tools/cfg5.py --rows 100000000 --cols 2000 --trees 1 --shard 0/8 > $OUT/set$i.log 2>&1
  rc=$?
  echo "set$i rc=$rc"
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
    print(c, "levels 0-5 (first fit):", " ".join(f"{v:.3g}" for v in vals[:6]))
PY
