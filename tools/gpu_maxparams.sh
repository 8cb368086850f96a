#!/bin/bash
# Param-offload GPU tests, a small Twin-Flow run, then the peak-trainable-params run (each step time-limited).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local t=$1; shift; echo "=== $* (limit ${t}s)"; timeout -k 10 "$t" "$@"; local rc=$?; echo "=== rc=$rc"; return $rc; }
step 300 python -u -m pytest tests/unit/runtime/test_zero_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/zero_gpu.log 2>&1 &&
step 300 python tools/bench_max_params.py --layers 4 --hidden 2048 --inter 5504 --heads 16 --ratio 0.5 > gpurun_out/maxparams_small.log 2>&1 &&
step 1000 python tools/bench_max_params.py ${MAXP_ARGS} > gpurun_out/maxparams.log 2>&1
echo "chain rc=$?"
