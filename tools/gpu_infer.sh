#!/bin/bash
# GPU check for the inference stack: all gpu-marked tests, the 7B decode benchmark, and (PROF="1 16") kernel profiles.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local t=$1; shift; echo "=== $* (limit ${t}s)"; timeout -k 10 "$t" "$@"; local rc=$?; echo "=== rc=$rc"; return $rc; }
step 900 python -m pytest tests/unit/ops tests/unit/inference tests/unit/runtime tests/unit/moe tests/unit/pipe tests/unit/sequence -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 || exit 1
step 600 python tools/bench_infer.py --batches ${BATCHES:-1,16,64} --prompt 512 --gen 64 > gpurun_out/bench_infer.log 2>&1 || exit 1
export TMPDIR=/tmp
for b in ${PROF:-}; do
  step 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_infer_b$b -o run --output-format csv -- python3 tools/bench_infer.py --batches $b --prompt 512 --gen 32 --graph 0 > gpurun_out/prof_infer_b$b.log 2>&1 || exit 1
done
echo "chain ok"
