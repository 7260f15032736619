set -o pipefail
mkdir -p gpurun_out/c3dbg
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --steps 10 --cpu-sample 0 --no-e2e > gpurun_out/c3dbg/c2.json 2> gpurun_out/c3dbg/c2.err || exit $?
AD_DEBUG_LEVELS=1 timeout -k 10 300 python3 -u bench.py --config C3 --steps 2 --warmup 1 --cpu-sample 0 --no-e2e > gpurun_out/c3dbg/c3.json 2> gpurun_out/c3dbg/c3.err || exit $?
echo ok
