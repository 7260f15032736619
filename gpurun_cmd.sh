set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_recovery.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_rec.log 2>&1
echo tests ok
