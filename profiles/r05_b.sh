set -o pipefail
O=gpurun_out/r05_b; mkdir -p $O
NO_BENCH=1 bash profiles/gpu_check.sh r05_b tests/test_gpu_sharding.py || exit $?
for N in 2 4; do
  timeout -k 10 400 python3 -u bench.py --gpus $N --transport host --steps 3 --warmup 1 --breakdown > $O/n${N}_bench.json 2> $O/n${N}_bench.err || { echo "n$N rc=$?"; tail -20 $O/n${N}_bench.err; exit 1; }
  cut -c1-300 $O/n${N}_bench.json
done
