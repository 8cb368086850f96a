#!/bin/bash
# 7B bench (default config) + rocprofv3 kernel-stats profile of a short run. Each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local t=$1; shift; echo "=== $* (limit ${t}s)"; timeout -k 10 "$t" "$@"; local rc=$?; echo "=== rc=$rc"; return $rc; }
step 600 python bench.py --steps ${STEPS:-5} --warmup 2 > gpurun_out/bench_7b.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof7b -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof7b.log 2>&1 || exit 1
echo "chain ok"
