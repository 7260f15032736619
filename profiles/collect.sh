#!/bin/bash
# profiles/collect.sh TAG — the round's measurement recipe, run on the GPU box from the repo root:
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash profiles/collect.sh r01_v2'
# 1. the default bench line (C2, with the CPU baseline leg) + its per-kernel HIP-event breakdown;
# 2. rocprofv3 --kernel-trace --stats of a short bench run (kernel durations to cross-check `roofline`);
# 3. two separate PMC passes (FETCH_SIZE, WRITE_SIZE — they do not fit one pass on gfx950), and the same two
#    for C3 and for C4 at the end;
# then, back in the build container (gpurun merges gpurun_out/ back):
#   python3 profiles/summarize.py gpurun_out/TAG TAG      -> profiles/TAG_*
# Every GPU step has its own time limit and the steps are chained (set -e): a failure ends the script.
set -eo pipefail
TAG=${1:?tag}
PART=${2:-all}          # c2: steps 1-4 only; c34: steps 5-7 only (two gpurun calls stay inside the call limit)
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
if [ "$PART" != "c34" ]; then
timeout -k 10 420 python3 -u "$ROOT/bench.py" --breakdown > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench done"
# (--no-e2e: the end-to-end side measurement overlaps PCIe uploads with pipelines, whose kernels then run slower
# than in the timed region; the stats must describe the timed region's kernels)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 3 --cpu-sample 0 --no-e2e --no-scaling-ref > "$OUT/stats.json" 2> "$OUT/stats.err"
echo "stats done"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-sample 0 --no-e2e --no-scaling-ref > "$OUT/fetch.log" 2>&1
echo "fetch done"
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-sample 0 --no-e2e --no-scaling-ref > "$OUT/write.log" 2>&1
echo "write done"
# 4. the CPU baseline's extrapolation check: the T-thread oracle once over the full C2 batch (NO_CPU_FULL=1 skips it)
[ -n "${NO_CPU_FULL:-}" ] || timeout -k 10 600 python3 -u "$ROOT/bench.py" --steps 3 --warmup 1 --cpu-sample 0 --no-e2e --cpu-full > "$OUT/cpu_full.json" 2> "$OUT/cpu_full.err"
echo "cpu full done"
fi
[ "$PART" = "c2" ] && exit 0
# 5. the other BASELINE configs on one GPU (secondary lines: C3 Zipf deep chains, C4 4M mixed key + range)
timeout -k 10 300 python3 -u "$ROOT/bench.py" --config C3 --steps 5 --warmup 2 --breakdown > "$OUT/c3.json" 2> "$OUT/c3.err"
echo "c3 done"
timeout -k 10 400 python3 -u "$ROOT/bench.py" --config C4 --steps 2 --warmup 1 --breakdown > "$OUT/c4.json" 2> "$OUT/c4.err"
echo "c4 done"
# 6. C3's PMC passes (the block level walk dominates it), separate counters as above
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c3fetch" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --config C3 --steps 1 --warmup 1 --cpu-sample 0 --no-e2e > "$OUT/c3fetch.log" 2>&1
echo "c3 fetch done"
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d "$OUT/c3write" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --config C3 --steps 1 --warmup 1 --cpu-sample 0 --no-e2e > "$OUT/c3write.log" 2>&1
echo "c3 write done"
# 7. C4's PMC passes (the virtual-item region dominates it)
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c4fetch" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --config C4 --steps 1 --warmup 1 --cpu-sample 0 --no-e2e > "$OUT/c4fetch.log" 2>&1
echo "c4 fetch done"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/c4write" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --config C4 --steps 1 --warmup 1 --cpu-sample 0 --no-e2e > "$OUT/c4write.log" 2>&1
echo "c4 write done"
