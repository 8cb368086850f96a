#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
step() { local t=$1; shift; echo "=== $* (limit ${t}s)"; timeout -k 10 "$t" "$@"; local rc=$?; echo "=== rc=$rc"; return $rc; }
step 900 python bench.py --steps 5 --warmup 2 --micro-batch 8 > gpurun_out/bench_7b_mb8.log 2>&1 &&
step 900 python bench.py --steps 5 --warmup 2 --micro-batch 6 > gpurun_out/bench_7b_mb6.log 2>&1
echo "chain rc=$?"
