set -o pipefail
O=gpurun_out/r05_ab; mkdir -p $O
NO_BENCH=1 bash profiles/gpu_check.sh r05_ab tests/test_gpu_block_levels.py tests/test_gpu_pipeline_union.py tests/test_golden.py tests/test_gpu_parity.py tests/test_gpu_history.py tests/test_gpu_stream.py || exit $?
timeout -k 10 300 python3 -u bench.py --config C3 --steps 5 --warmup 2 --cpu-sample 0 --no-e2e --no-scaling-ref --breakdown > $O/c3.json 2> $O/c3.err || { echo "c3 rc=$?"; tail -5 $O/c3.err; exit 1; }
grep "stages" $O/c3.err | cut -c1-200; cut -c1-200 $O/c3.json
timeout -k 10 300 python3 -u bench.py --steps 20 --cpu-sample 0 --no-e2e --no-scaling-ref > $O/c2.json 2> $O/c2.err || { echo "c2 rc=$?"; tail -5 $O/c2.err; exit 1; }
cut -c1-200 $O/c2.json
