#!/bin/bash
# Round-6: one PMC pass over the CV-loss kernel (enet_cvloss_gauss_kernel) in a short bench run
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_cvl}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $OUT/set1 -- \
    python3 $R/bench.py --steps 5 --warmup 1 --parity 0 --also-rct 0 --repeats 1 --inflight 1 > $OUT/set1.log 2>&1
rc=$?; echo "set1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 $R/tools/pmc_summary.py $OUT cvloss | tee $OUT/summary.txt
python3 - "$OUT" <<'PY'
import csv, glob, sys, statistics
d = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    d += [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f)) if "cvloss" in r["Kernel_Name"]]
print("cvloss traced us median", statistics.median(d), "n", len(d))
PY
