#!/bin/bash
# GPU check for the inference stack: all gpu-marked tests, then the 7B decode benchmark.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local t=$1; shift; echo "=== $* (limit ${t}s)"; timeout -k 10 "$t" "$@"; local rc=$?; echo "=== rc=$rc"; return $rc; }
step 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 &&
step 600 python tools/bench_infer.py --batches 1,16,64 --prompt 512 --gen 64 > gpurun_out/bench_infer.log 2>&1
echo "chain rc=$?"
