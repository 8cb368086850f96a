#!/bin/bash
# Full GPU gate: pytest -m gpu, smoke(), the default bench; each step time-limited.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local t=$1; shift; echo "=== $* (limit ${t}s)"; timeout -k 10 "$t" "$@"; local rc=$?; echo "=== rc=$rc"; return $rc; }
step 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r3_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r3_pytest_gpu.log
step 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { tail -30 gpurun_out/r3_smoke.log; exit 1; }
tail -1 gpurun_out/r3_smoke.log
step 500 python bench.py --steps ${STEPS:-10} --warmup 3 > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.log || { tail -30 gpurun_out/r3_bench.log; exit 1; }
cat gpurun_out/r3_bench.json
echo "chain ok"
