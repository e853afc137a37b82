#!/bin/bash
# (historical: drives the round-2..5 bench, whose --stagger flag was removed in round 6 when
#  the in-flight fits became the secondary "throughput_inflight" block)
# Bench step with / without cross-stream Gram staggering and over Gram workgroup counts,
# then a kernel trace of the default (staggered) step for tools/timeline.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
OUT=$R/gpurun_out/stagger.log
: > $OUT
one() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" timeout -k 10 300 python $R/bench.py --steps 20 --warmup 3 ${BARGS} > $R/gpurun_out/b_$tag.log 2>&1 || { echo "fail $tag"; tail -5 $R/gpurun_out/b_$tag.log; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step'],3), 'single', round(d['single_fit_ms'],3), repr(d['ate']), repr(d['se']))" $tag $R/gpurun_out/b_$tag.log | tee -a $OUT
}
for spec in ${SWEEP:-"1 1024 2 0" "1 1024 2 1" "2 2048 3 0" "2 2048 3 1" "2 1024 2 1" "2 4096 3 1"}; do
  set -- ${spec//,/ }
  BARGS="--stagger $1 --inflight $3 --blocked ${4:-1}" one s$1_wg$2_if$3_b${4:-1} ATE_GRAM_PAIR_WG=$2 || exit 1
done
[ -n "$NOPROF" ] && exit 0
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_stagger -o st \
  -- python3 $R/bench.py --steps 10 --warmup 2 ${PROF_ARGS} > $R/gpurun_out/prof_stagger.log 2>&1 || { echo prof failed; exit 1; }
python3 $R/tools/timeline.py $(find $R/gpurun_out/prof_stagger -name "*kernel_trace.csv") --window 40 | tee -a $OUT
