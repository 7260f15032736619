set -o pipefail
O=gpurun_out/r05_l; mkdir -p $O
NO_BENCH=1 bash profiles/gpu_check.sh r05_l tests/test_gpu_pipeline_union.py tests/test_golden.py tests/test_gpu_parity.py tests/test_gpu_block_levels.py tests/test_gpu_history.py tests/test_gpu_sharding.py || exit $?
timeout -k 10 200 python3 -u bench.py --steps 10 --cpu-sample 0 --no-scaling-ref --no-e2e --breakdown > $O/c2.json 2> $O/c2.err || { echo "c2 rc=$?"; tail -5 $O/c2.err; exit 1; }
grep "^  " $O/c2.err | head -16; cut -c1-200 $O/c2.json
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/stats" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 10 --warmup 3 --cpu-sample 0 --no-e2e --no-scaling-ref > "$R/$O/stats.json" 2> "$R/$O/stats.err" || exit 1
echo "stats done"
