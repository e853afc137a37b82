#!/bin/bash
# Round-6 full GPU check: the GPU suite on the production library, the suite on the debug
# library (load-time kernel resource check), then bench.py.
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"; shift
export TMPDIR=/tmp
step() { local n=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$n.log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] failed rc=$rc"; tail -30 "$OUT/$n.log"; exit $rc; fi
  echo "[$n] ok: $(tail -1 "$OUT/$n.log" | cut -c1-300)"; }
for s in "$@"; do
  case $s in
    tests) step tests 1200 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ;;
    testsall) step testsall 1200 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread ;;
    debugtests) ATE_DEBUG=1 step debugtests 1200 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ;;
    bench) step bench 400 python -u bench.py ;;
    smoke) step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    tests:*) step "tests_${s#tests:}" 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "${s#tests:}" ;;
  esac
done
