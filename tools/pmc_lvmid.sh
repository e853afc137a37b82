#!/bin/bash
# Round-6: PMC passes over the forest level engine's mid-node kernel (lv_mid_kernel) in the
# config-3 shard (tools/cfg3.py, 16 trees per forest, rank 0 of 8)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_lvmid}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "FETCH_SIZE TA_TA_BUSY_sum GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/set$i -- \
      python3 $R/tools/cfg3.py --rows 10000000 --cols 500 --trees 16 --shard 0/8 > $OUT/set$i.log 2>&1
  rc=$?
  echo "set$i rc=$rc"
  case $rc in 0) ;; *) tail -5 $OUT/set$i.log; exit $rc;; esac
done
python3 - "$OUT" <<'PY' | tee $OUT/summary.txt
import collections, csv, glob, sys
out = sys.argv[1]
tot = collections.defaultdict(float)
n = collections.defaultdict(int)
for f in glob.glob(out + "/**/*_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "lv_mid_kernel" not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]] += 1
dur = 0.0
nd = 0
for f in glob.glob(out + "/set1/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "lv_mid_kernel" in r["Kernel_Name"]:
            dur += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            nd += 1
print("lv_mid dispatches (set1)", nd, "total us", round(dur))
for c in sorted(tot):
    print(f"{c:28s} total {tot[c]:.4g} (n={n[c]})")
PY
