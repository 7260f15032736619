set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_range_index.py tests/test_gpu_recovery.py tests/test_gpu_max_conflicts.py tests/test_golden.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/t_ri.log 2>&1
echo tests1 ok
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "range or c4 or wide or merge_host" > gpurun_out/t_ri2.log 2>&1
echo tests2 ok
timeout -k 10 400 python3 -u bench.py --config C4 --steps 2 --warmup 1 --breakdown --cpu-sample 0 > gpurun_out/c4.json 2> gpurun_out/c4.err
echo c4 ok
