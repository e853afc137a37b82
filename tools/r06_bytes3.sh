#!/bin/bash
# Round-6: one-byte columns with the 16-byte two-half fragment layout -- byte GPU tests, tile
# kernel alone in both orders, the single call alternated, one PMC pass (LDS conflicts).
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local n=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$n.log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] failed rc=$rc"; tail -30 "$OUT/$n.log"; exit $rc; fi
  echo "[$n] ok: $(grep -E 'passed|failed|kernel|ms/call' "$OUT/$n.log" | tr '\n' ' ' | cut -c1-500)"; }
step tests 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "byte or gram"
ATE_GRAM_STAGE=tiles step gram_a 200 python -u tools/gram_only.py 1e7 pair pair16 pair pair16
ATE_GRAM_STAGE=tiles step gram_b 200 python -u tools/gram_only.py 1e7 pair16 pair pair16 pair
step single_ab 400 python -u tools/single_ab.py pair,pair16 4 20
R=$PWD
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d $R/$OUT/pmc1 -- python3 $R/tools/gram_only.py 1e7 pair pair16 pair pair16 > $R/$OUT/pmc1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d $R/$OUT/pmc2 -- python3 $R/tools/gram_only.py 1e7 pair pair16 pair pair16 > $R/$OUT/pmc2.log 2>&1 || exit $?
python3 $R/tools/pmc_summary.py $R/$OUT gram_bf16_pair
