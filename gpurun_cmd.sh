set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharding.py -m gpu -x -v --timeout 170 --timeout-method thread --durations=0 > gpurun_out/t_shr.log 2>&1
echo tests ok
