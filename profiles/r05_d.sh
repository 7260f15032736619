set -o pipefail
O=gpurun_out/r05_d; mkdir -p $O
NO_BENCH=1 TEST_LIMIT=800 bash profiles/gpu_check.sh r05_d tests || exit $?
timeout -k 10 200 python3 -u bench.py --steps 10 --cpu-sample 0 --no-scaling-ref --breakdown > $O/c2.json 2> $O/c2.err || { echo "c2 rc=$?"; tail -5 $O/c2.err; exit 1; }
cut -c1-300 $O/c2.json
timeout -k 10 200 python3 -u bench.py --config C3 --steps 5 --cpu-sample 0 --breakdown > $O/c3.json 2> $O/c3.err || { echo "c3 rc=$?"; tail -5 $O/c3.err; exit 1; }
cut -c1-300 $O/c3.json
