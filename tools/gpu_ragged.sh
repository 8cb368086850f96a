set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/unit/inference/test_paged_prefill_gpu.py tests/unit/inference/v2 tests/unit/ops/test_kernels_gpu.py -k "paged or ragged or qkv_rope" > gpurun_out/ragged_test.log 2>&1
