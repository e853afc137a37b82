# single-fit Gram round-count sweep (ATE_GRAM_ROUNDS): profiles/README r05 notes no change in 3-10 rounds
set -o pipefail
mkdir -p gpurun_out/r05_rounds
for r in 3 4 5 6 8 10; do
  ATE_GRAM_ROUNDS=$r timeout -k 10 200 python bench.py --steps 10 --warmup 2 --parity 0 --also-rct 0 > gpurun_out/r05_rounds/r$r.log 2>&1 || { echo fail $r; tail -5 gpurun_out/r05_rounds/r$r.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('rounds', sys.argv[2], 'ms/step', round(d['ms_per_step'],3), 'single', round(d['single_fit_ms'],3), d['single_fit_ms_all'])" gpurun_out/r05_rounds/r$r.log $r
done
