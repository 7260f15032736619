set -o pipefail
NO_BENCH=1 bash profiles/gpu_check.sh r05_c tests/test_cfk_store.py tests/test_gpu_cfk_release.py tests/test_reference_models.py tests/test_preaccept_expiry.py
