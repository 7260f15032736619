set -o pipefail
O=gpurun_out/r05_final; mkdir -p $O
NO_BENCH=1 TEST_LIMIT=1000 bash profiles/gpu_check.sh r05_final || exit $?
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/c3stats" -o run --output-format csv -- \
    python3 "$R/bench.py" --config C3 --steps 3 --warmup 1 --cpu-sample 0 --no-e2e --no-scaling-ref > "$R/$O/c3stats.json" 2> "$R/$O/c3stats.err" || exit 1
echo c3 stats done
