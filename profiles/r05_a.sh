set -o pipefail
mkdir -p gpurun_out/r05_a
NO_BENCH=1 bash profiles/gpu_check.sh r05_a tests/test_preaccept_expiry.py tests/test_gpu_block_levels.py tests/test_gpu_invert.py tests/test_gpu_cfk_release.py || exit $?
timeout -k 10 400 python3 -u bench.py --gpus 2 --transport host --steps 3 --warmup 1 --breakdown > gpurun_out/r05_a/n2_bench.json 2> gpurun_out/r05_a/n2_bench.err || { echo "n2 rc=$?"; tail -20 gpurun_out/r05_a/n2_bench.err; exit 1; }
cut -c1-600 gpurun_out/r05_a/n2_bench.json
