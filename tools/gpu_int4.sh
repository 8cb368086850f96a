#!/bin/bash
# int4 weight-only path: kernel tests, GEMV bench at Llama / BLOOM shapes, Llama-7B decode (bf16 vs int8 vs int4)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/unit/ops/test_int4_gemv.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tee gpurun_out/int4_pytest.log | tail -15 || exit 1
timeout -k 10 300 python -u tools/bench_int4_gemv.py ${QUICK:-} > gpurun_out/int4_gemv.jsonl 2> gpurun_out/int4_gemv.log || { tail -20 gpurun_out/int4_gemv.log; exit 1; }
cat gpurun_out/int4_gemv.jsonl
: > gpurun_out/llama7b_decode_int4.jsonl
for q in 0 8 4; do
  timeout -k 10 300 python -u tools/bench_infer.py --batches 1,8 --prompt 128 --gen 64 --graph 1 --quant-bits $q --group-size ${GS:-128} \
    >> gpurun_out/llama7b_decode_int4.jsonl 2> gpurun_out/llama7b_decode_q$q.log || { tail -20 gpurun_out/llama7b_decode_q$q.log; exit 1; }
done
cat gpurun_out/llama7b_decode_int4.jsonl
echo "chain ok"
