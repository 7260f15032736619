set -o pipefail
O=gpurun_out/r05_g; mkdir -p $O
NO_BENCH=1 bash profiles/gpu_check.sh r05_g tests/test_golden.py tests/test_gpu_parity.py tests/test_gpu_max_conflicts.py tests/test_gpu_history.py tests/test_gpu_block_levels.py tests/test_reference_models.py tests/test_gpu_invert.py || exit $?
timeout -k 10 200 python3 -u bench.py --steps 10 --cpu-sample 0 --no-scaling-ref --no-e2e --breakdown > $O/c2.json 2> $O/c2.err || { echo "c2 rc=$?"; tail -5 $O/c2.err; exit 1; }
grep "^  " $O/c2.err | head -16; cut -c1-200 $O/c2.json
