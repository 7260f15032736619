set -o pipefail
O=gpurun_out/r05_last; mkdir -p $O
bash profiles/gpu_check.sh r05_last tests/test_gpu_pipeline_union.py tests/test_cfk_store.py || exit $?
