set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/unit/ops/test_kernels_gpu.py -k "skinny_int8" > gpurun_out/i8_test.log 2>&1 && \
timeout -k 10 200 python -u tools/bench_int8_gemv.py > gpurun_out/i8_bench.jsonl 2>&1
