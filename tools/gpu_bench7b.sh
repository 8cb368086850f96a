#!/bin/bash
# 7B bench at two micro-batch sizes + a rocprofv3 kernel-stats profile of a short run.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local t=$1; shift; echo "=== $* (limit ${t}s)"; timeout -k 10 "$t" "$@"; local rc=$?; echo "=== rc=$rc"; return $rc; }
step 900 python bench.py --steps 4 --warmup 2 --micro-batch 2 > gpurun_out/bench_7b_mb2.log 2>&1 &&
step 900 python bench.py --steps 4 --warmup 2 --micro-batch 4 > gpurun_out/bench_7b_mb4.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
step 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof7b -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --micro-batch 2 > gpurun_out/prof7b.log 2>&1
echo "chain rc=$?"
