set -o pipefail
O=gpurun_out/r05_x; mkdir -p $O
NO_BENCH=1 bash profiles/gpu_check.sh r05_x tests/test_gpu_pipeline_union.py tests/test_golden.py tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_history.py tests/test_gpu_sharding.py tests/test_gpu_accept.py tests/test_gpu_max_conflicts.py || exit $?
timeout -k 10 300 python3 -u bench.py --steps 20 --cpu-sample 0 --no-scaling-ref > $O/c2.json 2> $O/c2.err || { echo "c2 rc=$?"; tail -5 $O/c2.err; exit 1; }
cut -c1-200 $O/c2.json
