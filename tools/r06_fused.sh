#!/bin/bash
# Round-6: fused root histogram of a fold's two GBDT fits (csrc/gbdt.hip gbdt_hist2_kernel) --
# GPU GBDT tests, then the config-5 shard (10 trees per model) fused vs one fit after the
# other, alternated, then a kernel trace of each.
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"; T=${2:-10}
export TMPDIR=/tmp
step() { local n=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$n.log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] failed rc=$rc"; tail -30 "$OUT/$n.log"; exit $rc; fi
  echo "[$n] ok: $(tail -1 "$OUT/$n.log" | cut -c1-400)"; }
step tests 400 python -u -m pytest tests/test_gbdt_gpu.py -x -q --timeout 200 --timeout-method thread
for i in 1 2; do
  ATE_GBDT_FUSED_ROOT=1 step cfg5_fused_$i 300 python -u tools/cfg5.py --rows 1e8 --cols 2000 --trees $T --shard 0/8
  ATE_GBDT_FUSED_ROOT=0 step cfg5_serial_$i 300 python -u tools/cfg5.py --rows 1e8 --cols 2000 --trees $T --shard 0/8
done
R=$PWD
cd /tmp
for v in 1 0; do
  ATE_GBDT_FUSED_ROOT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_$v -- python3 $R/tools/cfg5.py --rows 1e8 --cols 2000 --trees $T --shard 0/8 > $R/$OUT/prof_$v.log 2>&1 || exit $?
done
echo profiled
