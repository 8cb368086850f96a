set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/unit/ops/test_kernels_gpu.py -k "skinny_int8" > gpurun_out/i8_test.log 2>&1 && \
BATCHES=1,16 bash tools/gpu_bloom.sh
