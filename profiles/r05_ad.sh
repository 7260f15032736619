set -o pipefail
O=gpurun_out/r05_ad; mkdir -p $O
NO_BENCH=1 bash profiles/gpu_check.sh r05_ad tests/test_gpu_pipeline_union.py tests/test_golden.py tests/test_gpu_parity.py tests/test_gpu_block_levels.py tests/test_gpu_stream.py tests/test_gpu_history.py tests/test_gpu_fullsize.py || exit $?
for mode in fused plain fused plain; do
  if [ $mode = plain ]; then export AD_NO_FUSED_CHAINS=1; else unset AD_NO_FUSED_CHAINS; fi
  timeout -k 10 300 python3 -u bench.py --steps 30 --cpu-sample 0 --no-e2e --no-scaling-ref > $O/c2_$mode.json 2> $O/c2_$mode.err || { echo "c2 rc=$?"; tail -5 $O/c2_$mode.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c2_$mode.json').read().strip().splitlines()[-1]); print('$mode', d['ms_per_step'], d['pipeline']['frac'], d['pipeline']['stage_ms'])"
done
