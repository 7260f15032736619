set -o pipefail
O=gpurun_out/r05_e; mkdir -p $O
NO_BENCH=1 bash profiles/gpu_check.sh r05_e tests/test_reference_models.py tests/test_wire.py tests/test_gpu_sharding.py || exit $?
timeout -k 10 200 python3 -u bench.py --steps 10 --cpu-sample 0 --no-scaling-ref --breakdown > $O/c2.json 2> $O/c2.err || { echo "c2 rc=$?"; tail -5 $O/c2.err; exit 1; }
cut -c1-300 $O/c2.json
timeout -k 10 200 python3 -u bench.py --config C3 --steps 5 --cpu-sample 0 --breakdown > $O/c3.json 2> $O/c3.err || { echo "c3 rc=$?"; tail -5 $O/c3.err; exit 1; }
cut -c1-300 $O/c3.json
timeout -k 10 400 python3 -u bench.py --gpus 2 --transport host --steps 3 --warmup 1 > $O/n2.json 2> $O/n2.err || { echo "n2 rc=$?"; tail -5 $O/n2.err; exit 1; }
cut -c1-300 $O/n2.json
