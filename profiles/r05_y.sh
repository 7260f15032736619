set -o pipefail
O=gpurun_out/r05_y; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/stats" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 10 --warmup 3 --cpu-sample 0 --no-e2e --no-scaling-ref > "$R/$O/stats.json" 2> "$R/$O/stats.err"
echo stats done
