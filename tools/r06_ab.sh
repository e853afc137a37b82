#!/bin/bash
# Round-6 A/B session: gram kernel alone (tri vs pair), then bench.py with each.
#   bash tools/r06_ab.sh OUT
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local n=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$n.log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] failed rc=$rc"; tail -30 "$OUT/$n.log"; exit $rc; fi
  echo "[$n] ok: $(tail -1 "$OUT/$n.log" | cut -c1-300)"; }
step tests 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "gram or dml or lasso"
ATE_GRAM_STAGE=tiles step gram_tiles 200 python -u tools/gram_only.py 1e7 pair tri pair tri
step gram_all 200 python -u tools/gram_only.py 1e7 pair tri
ATE_GRAM_TRI=0 step bench_pair 300 python -u bench.py --also-rct 0
step bench_tri 300 python -u bench.py --also-rct 0
python - "$OUT" <<'PY'
import json, sys
for n in ("bench_pair", "bench_tri"):
    d = json.loads(open(f"{sys.argv[1]}/{n}.log").read().strip().splitlines()[-1])
    print(n, "ms/step", round(d["ms_per_step"], 3), "single", round(d["single_fit_ms"], 3),
          "inflight", round(d["throughput_inflight"]["ms_per_fit"], 3), d["ate_hex"], d["se_hex"],
          "parity", d["parity"]["abs_diff_ate_in_se"])
PY
