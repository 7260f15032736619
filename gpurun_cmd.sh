set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_history.py tests/test_gpu_max_conflicts.py tests/test_wire.py tests/test_gpu_sharding.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_hist.log 2>&1
echo tests ok
