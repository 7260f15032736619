set -o pipefail
O=gpurun_out/r05_ht; mkdir -p $O
AD_HOST_TIMERS=1 timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 3 --cpu-sample 0 --no-e2e --no-scaling-ref > $O/c2.json 2> $O/c2.err || { echo "rc=$?"; tail -5 $O/c2.err; exit 1; }
grep host_timers $O/c2.err | tail -4
