#!/bin/bash
# One parameterised GPU-box session (replaces the per-session tools/gpu_r0*.sh scripts).
#
#   bash tools/gpu_session.sh OUT step [step ...]        (run by gpurun from the repo root)
#
# Every step runs under its own time limit; the session stops at the first failure
# (a GPU fault / abort / time limit ends it: nothing more runs on the GPU). Outputs go to
# gpurun_out/OUT/. Steps:
#   tests          the whole GPU suite (pytest -m gpu)
#   tests:EXPR     GPU tests selected by -k EXPR
#   debugtests     the GPU suite on the device-assertion build (ATE_DEBUG=1, _build.py)
#   smoke          __graft_entry__.smoke()
#   bench          bench.py (driver defaults), one JSON line
#   prof           rocprofv3 kernel trace + stats of a short bench, and the overlap timeline
#   enet_ab:A,B,.. CV-LASSO stage alone for libatehip_<A>.so, ... ("new" = in-tree), x2
#   enet_prof      cycle accounting of the path kernel (tools/enet_profile.py build)
#   gram_ab:A,B,.. the bf16 Gram tile kernel alone (tools/gram_only.py) per library, x2
#   cfg4           config 4 (tools/cfg4.py): one GPU, then rank 0 of 8 alone; cfg4phases: phase timing
#   cfg3           config-3 per-GPU shard (N=1e7, p=500, 100 trees, rank 0 of 8)
#   cfg5           config-5 per-GPU shard (N=1.25e7, p=2000, 100 trees); cfg5c: concurrent Y/W fits
#   cfg5small      a small config-5 shard, concurrent then serial Y/W fits
#   c04_ab         a small config-5 shard: feature-sliced C04 vs ATE_GBDT_C04=allreduce, x2
#   micro          tools/micro/mfma_peak (matrix / vector peaks) and the fp64 Gram alone
#   lvgaps         idle gaps of the host-driven forest level engine (kernel trace)
#   single         kernel trace of bench.py: the last single-fit replay's critical path
#   ktrace_ab:A,B[:RX] kernel trace of bench.py per library (ATE_HIP_LIB), mean time of RX kernels
#   configs        all BASELINE configs on one GPU (tools/bench_configs.py)
#   replicate      the 14-row tutorial driver, warm timing (tools/replicate_timing.py)
#   gramdump       the bench panel's fold Gram stack -> OUT/gram_dump (tools/dump_bench_gram.py)
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
ROOT=$(pwd)
export TMPDIR=/tmp

run() {   # run NAME LIMIT CMD...: time-limited step, log to $OUT/NAME.log, stop on failure
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "[$name] failed rc=$rc"; tail -25 "$OUT/$name.log"; exit $rc
  fi
  echo "[$name] ok: $(tail -1 "$OUT/$name.log" | cut -c1-400)"
}

for step in "$@"; do
  case $step in
    tests)
      run tests 1500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ;;
    tests:*)
      run "tests_${step#tests:}" 900 python -u -m pytest tests -m gpu -x -v --timeout 240 \
          --timeout-method thread -k "${step#tests:}" ;;
    libtests:*)  # libtests:NAME:EXPR -- GPU tests -k EXPR on _lib/libatehip_NAME.so
      spec=${step#libtests:}; nm=${spec%%:*}; ex=${spec#*:}
      ATE_HIP_LIB=$ROOT/ate_replication_causalml_amd/_lib/libatehip_$nm.so \
        run "libtests_$nm" 900 python -u -m pytest tests -m gpu -x -q --timeout 240 \
          --timeout-method thread -k "$ex" ;;
    debugtests)
      ATE_DEBUG=1 run debugtests 1500 python -u -m pytest tests -m gpu -x -q --timeout 240 \
          --timeout-method thread ;;
    smoke)
      run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      run bench 300 python bench.py ;;
    bench_ab:*)  # bench_ab:A,B,.. -- bench.py on each _lib/libatehip_<A>.so ("new" = in-tree)
      IFS=, read -ra libs <<< "${step#bench_ab:}"
      for nm in "${libs[@]}"; do
        lib=ate_replication_causalml_amd/_lib/libatehip_$nm.so
        [ "$nm" = new ] && lib=ate_replication_causalml_amd/_lib/libatehip.so
        ATE_HIP_LIB=$ROOT/$lib run "bench_$nm" 300 python bench.py || exit 1
      done ;;
    prof)
      ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$ROOT/$OUT/prof" -o bench -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --also-rct 0 \
          > "$ROOT/$OUT/prof.log" 2>&1 ) || { echo "[prof] failed"; tail -20 "$OUT/prof.log"; exit 1; }
      python3 -c "import sys; sys.path.insert(0, 'tools'); import timeline; timeline.overlapped(sys.argv[1], 24)" \
          $(find "$OUT/prof" -name "*kernel_trace.csv") > "$OUT/prof_timeline.txt" 2>&1 || true
      echo "[prof] ok" ;;
    enet_ab:*)
      IFS=, read -ra libs <<< "${step#enet_ab:}"
      for rep in 1 2; do
        for nm in "${libs[@]}"; do
          lib=ate_replication_causalml_amd/_lib/libatehip_$nm.so
          [ "$nm" = new ] && lib=ate_replication_causalml_amd/_lib/libatehip.so
          ATE_HIP_LIB=$ROOT/$lib run "enet_${nm}_$rep" 120 python tools/enet_only.py 15
        done
      done ;;
    gram_ab:*)
      IFS=, read -ra libs <<< "${step#gram_ab:}"
      for rep in 1 2; do
        for nm in "${libs[@]}"; do
          lib=ate_replication_causalml_amd/_lib/libatehip_$nm.so
          [ "$nm" = new ] && lib=ate_replication_causalml_amd/_lib/libatehip.so
          ATE_HIP_LIB=$ROOT/$lib ATE_GRAM_STAGE=tiles run "gram_${nm}_$rep" 120 python tools/gram_only.py
        done
      done ;;
    enet_prof)
      run enet_prof 300 python tools/enet_profile.py ;;
    enet_prof_rct)
      ATE_DGP=rct run enet_prof_rct 300 python tools/enet_profile.py ;;
    enet_clock)  # path kernel clock alone vs beside a Gram (tools/enet_profile.py --build first)
      run enet_clock 200 python -u tools/enet_clock.py && \
      ATE_DGP=rct run enet_clock_rct 200 python -u tools/enet_clock.py ;;
    cfg4)        # config 4 on one GPU (all trees, all replicates) and rank 0's share of 8
      run cfg4 300 python -u tools/cfg4.py --rows 50000 && \
      run cfg4_shard 300 python -u tools/cfg4.py --rows 50000 --shard 0/8 ;;
    cfg4phases)
      run cfg4phases 300 python -u tools/cfg4_phases.py ;;
    xprof)       # phase ticks of one exact-split grf causal tree (tools/exact_forest_prof.py --build first)
      run xprof 200 python -u tools/exact_forest_prof.py --causal ;;
    cfg3)
      run cfg3 300 python -u tools/cfg3.py --rows 10000000 --cols 500 --trees 100 --shard 0/8 ;;
    cfg5)
      run cfg5 400 python -u tools/cfg5.py --rows 100000000 --cols 2000 --trees 100 --shard 0/8 ;;
    cfg5c)
      run cfg5c 400 python -u tools/cfg5.py --rows 100000000 --cols 2000 --trees 100 --shard 0/8 --concurrent ;;
    cfg5small)   # 1/8 of a shard: both orders, same bits
      run cfg5small_c 200 python -u tools/cfg5.py --rows 12500000 --cols 2000 --trees 20 --shard 0/8 --concurrent && \
      run cfg5small_s 200 python -u tools/cfg5.py --rows 12500000 --cols 2000 --trees 20 --shard 0/8 ;;
    c04_ab)      # 1/8 of a shard, feature-sliced C04 (default at --shard 0/8) vs all-reduce, x2
      for rep in 1 2; do
        run c04_sliced_$rep 200 python -u tools/cfg5.py --rows 12500000 --cols 2000 --trees 20 --shard 0/8 && \
        ATE_GBDT_C04=allreduce run c04_allreduce_$rep 200 python -u tools/cfg5.py --rows 12500000 \
          --cols 2000 --trees 20 --shard 0/8 || exit 1
      done ;;
    micro)       # MFMA / vector FMA peaks and the fp64 Gram alone
      run mfma_peak 60 ./tools/micro/mfma_peak && \
      run gram_f64 200 python -u tools/gram_f64_time.py ;;
    lvgaps)      # one config-3 forest on the level engine under a kernel trace: idle gaps
      ( cd /tmp && ENGINES=level timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
          -d "$ROOT/$OUT/lvprof" -o lv -- python3 "$ROOT/tools/forest_level_probe.py" \
          > "$ROOT/$OUT/lvgaps_run.log" 2>&1 ) || { echo "[lvgaps] failed"; tail -20 "$OUT/lvgaps_run.log"; exit 1; }
      python3 tools/gap_summary.py $(find "$OUT/lvprof" -name "*kernel_trace.csv") lv_ \
          > "$OUT/lvgaps.txt" 2>&1
      echo "[lvgaps] ok: $(cat "$OUT/lvgaps.txt")"
      ENGINES=level run lvplain 200 python -u tools/forest_level_probe.py ;;
    single)      # kernel trace of bench.py: the last single-fit replay's critical path
      ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
          -d "$ROOT/$OUT/single" -o single -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 \
          --parity 0 --also-rct 0 --dgp "${ATE_DGP:-tutorial}" > "$ROOT/$OUT/single_run.log" 2>&1 ) || { echo "[single] failed"; tail -20 "$OUT/single_run.log"; exit 1; }
      python3 tools/single_fit_timeline.py $(find "$OUT/single" -name "*kernel_trace.csv") \
          > "$OUT/single_timeline.txt" 2>&1
      echo "[single] ok: $(tail -14 "$OUT/single_timeline.txt")" ;;
    ktrace_ab:*) # ktrace_ab:A,B,..[:REGEX] kernel-trace bench.py per library, mean time of REGEX kernels
      spec=${step#ktrace_ab:}; IFS=: read -r libs_csv rx <<< "$spec"; rx=${rx:-enet_cvloss}
      IFS=, read -ra libs <<< "$libs_csv"
      for nm in "${libs[@]}"; do
        lib=ate_replication_causalml_amd/_lib/libatehip_$nm.so
        [ "$nm" = new ] && lib=ate_replication_causalml_amd/_lib/libatehip.so
        ( cd /tmp && ATE_HIP_LIB=$ROOT/$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
            -d "$ROOT/$OUT/kt_$nm" -o kt -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --parity 0 --also-rct 0 \
            > "$ROOT/$OUT/kt_$nm.log" 2>&1 ) || { echo "[kt_$nm] failed"; tail -20 "$OUT/kt_$nm.log"; exit 1; }
        python3 -c "
import csv, re, sys, statistics as st
r = [x for x in csv.DictReader(open(sys.argv[1])) if re.search(sys.argv[2], x['Kernel_Name'])]
d = [(int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1e3 for x in r]
print(sys.argv[3], len(d), 'kernels, mean %.1f us, median %.1f us' % (st.mean(d), st.median(d)))
" $(find "$OUT/kt_$nm" -name "*kernel_trace.csv") "$rx" "$nm" | tee -a "$OUT/ktrace_ab.txt"
      done ;;
    configs)
      run configs 900 python -u tools/bench_configs.py ;;
    replicate)
      run replicate 600 python -u tools/replicate_timing.py ;;
    replicate:*) # replicate:NAME -- the same passes on _lib/libatehip_NAME.so
      nm=${step#replicate:}
      ATE_HIP_LIB=$ROOT/ate_replication_causalml_amd/_lib/libatehip_$nm.so \
        run "replicate_$nm" 600 python -u tools/replicate_timing.py ;;
    gramdump)    # the bench panel's fold Gram stack for tools/enet_sim.py
      run gramdump 200 python -u tools/dump_bench_gram.py "$OUT/gram_dump" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
