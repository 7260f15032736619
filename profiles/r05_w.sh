set -o pipefail
O=gpurun_out/r05_w; mkdir -p $O
NO_BENCH=1 bash profiles/gpu_check.sh r05_w tests/test_gpu_block_levels.py tests/test_golden.py tests/test_gpu_history.py || exit $?
timeout -k 10 300 python3 -u bench.py --config C3 --steps 5 --warmup 2 --cpu-sample 0 --no-e2e --no-scaling-ref --breakdown > $O/c3.json 2> $O/c3.err || { echo "c3 rc=$?"; tail -5 $O/c3.err; exit 1; }
grep "^  " $O/c3.err | head -3; cut -c1-200 $O/c3.json
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$R/$O/c3fetch" -o run --output-format csv -- \
    python3 "$R/bench.py" --config C3 --steps 1 --warmup 1 --cpu-sample 0 --no-e2e --no-scaling-ref > "$R/$O/c3fetch.log" 2>&1 || exit 1
echo "c3 fetch done"
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d "$R/$O/c3write" -o run --output-format csv -- \
    python3 "$R/bench.py" --config C3 --steps 1 --warmup 1 --cpu-sample 0 --no-e2e --no-scaling-ref > "$R/$O/c3write.log" 2>&1 || exit 1
echo "c3 write done"
