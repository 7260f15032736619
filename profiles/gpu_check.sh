#!/bin/bash
# profiles/gpu_check.sh TAG [pytest targets...] — the round's GPU check recipe, run on the GPU box from the repo root:
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash profiles/gpu_check.sh r04_x tests/test_gpu_invert.py'
# 1. the -m gpu tests given (default: all), one process, per-test timeout; 2. smoke(); 3. a short default bench line.
# Each GPU step has its own time limit; a fault / abort / time limit ends the script (test failures alone do not).
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
rc=0
[ $# -gt 0 ] || set -- tests
timeout -k 10 ${TEST_LIMIT:-900} python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" \
    > "$OUT/tests.log" 2>&1 || rc=$?
echo "tests rc=$rc"; tail -3 "$OUT/tests.log"
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
echo smoke ok
if [ -z "$NO_BENCH" ]; then
    timeout -k 10 300 python3 -u bench.py --steps 10 --cpu-sample 0 --breakdown > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
    echo bench ok; cat "$OUT/bench.json" | cut -c1-400
fi
exit $rc
