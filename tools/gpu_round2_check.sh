#!/bin/bash
# Round-2 check after the ZeRO-3 reuse-distance change: ZeRO GPU tests, the 7B forced-partition bench (full multi-rank
# code path on one GPU: partitioned groups, RCCL all-gather / reduce-scatter), the default bench, and the flash-bwd
# ablation of the shipped (atomic dQ) kernel. Each step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local t=$1; shift; echo "=== $* (limit ${t}s)"; timeout -k 10 "$t" "$@"; local rc=$?; echo "=== rc=$rc"; return $rc; }
step 300 python -u -m pytest tests/unit/runtime/test_zero_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/zero_gpu.log 2>&1 || exit 1
step 600 env DS_ZERO_FORCE_PARTITION=1 python bench.py --steps 6 --warmup 2 > gpurun_out/forced_bench.log 2>&1 || exit 1
step 600 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_7b.log 2>&1 || exit 1
step 200 python tools/flash_bwd_ablate.py > gpurun_out/ablate_atomic.log 2>&1 || exit 1
echo "chain ok"
