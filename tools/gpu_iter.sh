#!/bin/bash
# Iteration check: kernel tests, 7B bench (MB=4), kernel-stats profile (MB=2, 2 steps).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local t=$1; shift; echo "=== $* (limit ${t}s)"; timeout -k 10 "$t" "$@"; local rc=$?; echo "=== rc=$rc"; return $rc; }
step 600 python -m pytest tests/unit/ops -m gpu -q > gpurun_out/pytest_gpu.log 2>&1 &&
step 900 python bench.py --steps 5 --warmup 2 --micro-batch ${MB:-4} > gpurun_out/bench_7b.log 2>&1 &&
export TMPDIR=/tmp &&
step 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof7b -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --micro-batch 2 > gpurun_out/prof7b.log 2>&1
echo "chain rc=$?"
