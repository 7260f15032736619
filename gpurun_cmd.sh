set -o pipefail
D=gpurun_out/${TAG:-r03e}
mkdir -p $D
export TMPDIR=/tmp
rc=0
timeout -k 10 1000 python3 -u -m pytest --maxfail=15 -v --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests} > $D/tests.log 2>&1 || rc=$?
echo "tests rc=$rc"
# 1 = some tests failed (the GPU is fine); anything else (timeout, abort, fault) ends the call here
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit $?
echo smoke ok
timeout -k 10 300 python3 -u bench.py --steps 10 --cpu-sample 0 --breakdown > $D/bench.json 2> $D/bench.err || exit $?
echo bench ok
exit $rc
