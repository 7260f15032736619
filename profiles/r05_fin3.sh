# r05_fin3: the k_radix_hist change (16-byte loads of full tiles) -- parity tests that cover the Params it
# produces (every stage derives its packing from them), then C2 bench lines and a rocprof stats pass
set -o pipefail
O=gpurun_out/r05_fin3; mkdir -p $O
NO_BENCH=1 TEST_LIMIT=600 bash profiles/gpu_check.sh r05_fin3 tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_pipeline_union.py tests/test_gpu_fullsize.py tests/test_gpu_range_index.py || exit $?
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 30 --cpu-sample 0 --no-e2e --no-scaling-ref > $O/c2_$i.json 2> $O/c2_$i.err || { echo "c2 rc=$?"; tail -5 $O/c2_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/c2_$i.json').read().strip().splitlines()[-1]); print('c2', d['ms_per_step'])"
done
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/stats" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 10 --warmup 3 --cpu-sample 0 --no-e2e --no-scaling-ref > "$R/$O/stats.json" 2> "$R/$O/stats.err"
echo stats done
