set -eo pipefail
mkdir -p gpurun_out/r03d
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_stream.py tests/test_gpu_cfk_state.py tests/test_gpu_history.py tests/test_gpu_accept.py tests/test_gpu_parity.py tests/test_gpu_sharding.py > gpurun_out/r03d/tests.log 2>&1
echo tests ok
timeout -k 10 300 python3 -u bench.py --steps 10 --cpu-sample 0 --breakdown > gpurun_out/r03d/bench.json 2> gpurun_out/r03d/bench.err
echo bench ok
