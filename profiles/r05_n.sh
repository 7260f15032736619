set -o pipefail
O=gpurun_out/r05_n; mkdir -p $O
AD_HOST_TIMERS=1 timeout -k 10 200 python3 -u bench.py --steps 6 --warmup 2 --cpu-sample 0 --no-scaling-ref --no-e2e > $O/c2.json 2> $O/c2.err || { echo "c2 rc=$?"; tail -5 $O/c2.err; exit 1; }
grep host_timers $O/c2.err | tail -4; cut -c1-200 $O/c2.json
