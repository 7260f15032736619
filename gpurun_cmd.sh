set -eo pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_block_levels.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_rev.log 2>&1
echo tests ok
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-sample 0 > gpurun_out/b_rev.json 2> gpurun_out/b_rev.err
timeout -k 10 400 python -u bench.py --config C4 --steps 2 --warmup 1 --cpu-sample 0 --breakdown > gpurun_out/b_rev_c4.json 2> gpurun_out/b_rev_c4.err
echo bench ok
