#!/bin/bash
# profiles/trace.sh TAG [bench args...] — kernel trace + stats of a short bench run only (the quick loop between
# full profiles/collect.sh runs):  gpurun -- 'bash profiles/trace.sh r03_x'
# then: python3 profiles/timeline.py gpurun_out/TAG   (one step's dispatch sequence with gaps)
set -eo pipefail
TAG=${1:?tag}
shift
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 3 --cpu-sample 0 --no-e2e "$@" > "$OUT/stats.json" 2> "$OUT/stats.err"
echo "trace done"
