set -eo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err
echo bench ok
