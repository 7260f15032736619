set -eo pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_accept.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_vi.log 2>&1
echo tests ok
timeout -k 10 500 python -u bench.py --config C4 --steps 3 --warmup 1 --cpu-sample 0 --breakdown > gpurun_out/b_vi_c4.json 2> gpurun_out/b_vi_c4.err
echo bench ok
