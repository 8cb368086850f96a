#!/bin/bash
# Round-2 batch 2: MoE / random-LTD kernel tests (token sort), the long-context point of BASELINE config 3
# (Llama-2-7B, seq 32768, 1 GPU), and a kernel-stats profile of the current 7B step. Each step has its own limit.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local t=$1; shift; echo "=== $* (limit ${t}s)"; timeout -k 10 "$t" "$@"; local rc=$?; echo "=== rc=$rc"; return $rc; }
step 300 python -u -m pytest tests/unit/ops/test_moe_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/moe_gpu.log 2>&1 || exit 1
step 600 python bench.py --seq-len 32768 --micro-batch 1 --steps 4 --warmup 2 > gpurun_out/bench_7b_32k.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof7b -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof7b.log 2>&1 || exit 1
echo "chain ok"
