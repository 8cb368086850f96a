#!/bin/bash
# Flash backward: GPU numerics tests (dense, causal, GQA, block-sparse), the bench vs the library kernel, the ablation.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/unit/ops/test_flash_attn_gpu.py tests/unit/ops/sparse_attention tests/unit/sequence -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fb_tests.log 2>&1 &&
timeout -k 10 300 python tools/bench_flash_bwd.py > gpurun_out/fb_bench.log 2>&1 &&
timeout -k 10 200 python tools/flash_bwd_ablate.py > gpurun_out/ablate.log 2>&1
echo rc=$?
