# r05_fin5: the final round-5 code (k_minmax back to 1024 blocks + a 256-thread fold, 16-byte key loads kept) -- the whole -m gpu suite, smoke, the default
# bench line, then a rocprof stats pass of the C2 timed region
set -o pipefail
O=gpurun_out/r05_fin5; mkdir -p $O
TEST_LIMIT=600 bash profiles/gpu_check.sh r05_fin5 tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_pipeline_union.py tests/test_gpu_stream.py || exit $?
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/stats" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 10 --warmup 3 --cpu-sample 0 --no-e2e --no-scaling-ref > "$R/$O/stats.json" 2> "$R/$O/stats.err"
echo stats done
