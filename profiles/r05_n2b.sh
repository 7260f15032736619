set -o pipefail
O=gpurun_out/r05_n2b; mkdir -p $O
timeout -k 10 500 python3 -u bench.py --gpus 2 --transport host --steps 3 --warmup 1 > $O/n2.json 2> $O/n2.err || { echo "n2 rc=$?"; tail -20 $O/n2.err; exit 1; }
cut -c1-300 $O/n2.json
