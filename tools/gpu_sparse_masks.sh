#!/bin/bash
# block-sparse attention with in-kernel masks: tests, then the masked-vs-unmasked bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/unit/ops/sparse_attention tests/unit/ops/test_flash_attn_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tee gpurun_out/sparse_masks_pytest.log | tail -15 || exit 1
timeout -k 10 300 python -u tools/bench_sparse_attn.py > gpurun_out/sparse_attn_bench.jsonl 2> gpurun_out/sparse_attn_bench.log || { tail -20 gpurun_out/sparse_attn_bench.log; exit 1; }
cat gpurun_out/sparse_attn_bench.jsonl
echo "chain ok"
