# r05_fin4: the final round-5 code (k_minmax_final over 1024 threads) -- the whole -m gpu suite, smoke, the default
# bench line, then a rocprof stats pass of the C2 timed region
set -o pipefail
O=gpurun_out/r05_fin4; mkdir -p $O
TEST_LIMIT=600 bash profiles/gpu_check.sh r05_fin4 tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_pipeline_union.py tests/test_gpu_stream.py || exit $?
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/stats" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 10 --warmup 3 --cpu-sample 0 --no-e2e --no-scaling-ref > "$R/$O/stats.json" 2> "$R/$O/stats.err"
echo stats done
