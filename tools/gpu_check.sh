#!/bin/bash
# One GPU session: kernel numerics tests, smoke, small bench, 7B bench. Each GPU step has its own time limit and
# the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local t=$1; shift; echo "=== $* (limit ${t}s)"; timeout -k 10 "$t" "$@"; local rc=$?; echo "=== rc=$rc"; return $rc; }
step 600 python -m pytest tests/unit/ops -m gpu -q > gpurun_out/pytest_gpu.log 2>&1 &&
step 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
step 300 python bench.py --model tiny --steps 5 --warmup 2 --micro-batch 4 --seq-len 2048 > gpurun_out/bench_tiny.log 2>&1 &&
step 900 python bench.py --steps 4 --warmup 2 --micro-batch ${MB:-2} > gpurun_out/bench_7b.log 2>&1
echo "chain rc=$?"
