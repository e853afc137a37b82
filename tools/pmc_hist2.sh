#!/bin/bash
# Round-6 PMC passes over the fused root histogram kernel (gbdt_hist2_kernel) (tools/cfg5.py, per-GPU shard
# N=1.25e7 x p=2000 tutorial panel, one tree per model): LDS array activity and atomics,
# VALU, TA, HBM fetch -- one counter set per rocprofv3 run (each within the per-block slot
# limits), every pass under its own kill timeout.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_hist2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/set$i -- \
      python3 $R/tools/cfg5.py --rows 100000000 --cols 2000 --trees 1 --shard 0/8 > $OUT/set$i.log 2>&1
  rc=$?
  echo "set$i ($set) rc=$rc"
  case $rc in 0) ;; *) tail -5 $OUT/set$i.log; exit $rc;; esac
done
python3 - "$OUT" <<'PY' | tee $OUT/summary.txt
import collections, csv, glob, sys
out = sys.argv[1]
per = collections.defaultdict(lambda: collections.defaultdict(float))
dur = {}
for f in glob.glob(out + "/**/*_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gbdt_hist2_kernel" not in r["Kernel_Name"]:
            continue
        per[r["Counter_Name"]][(f, int(r["Dispatch_Id"]))] += float(r["Counter_Value"])
for f in glob.glob(out + "/**/*kernel_trace.csv", recursive=True):
    ks = [r for r in csv.DictReader(open(f)) if "gbdt_hist2_kernel" in r["Kernel_Name"]]
    dur[f] = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ks]
for f, d in dur.items():
    print("fused root dispatches", len(d), "us:", " ".join(f"{v:.0f}" for v in d[:7]))
for c, d in sorted(per.items()):
    vals = [v for _, v in sorted(d.items(), key=lambda kv: kv[0][1])]
    print(f"{c:34s} fused root, per dispatch: " + " ".join(f"{v:.4g}" for v in vals[:5]))
PY
