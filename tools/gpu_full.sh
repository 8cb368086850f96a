#!/bin/bash
# Round check: every gpu-marked test, the graft smoke, and the 7B ZeRO-3 training bench (default config).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local t=$1; shift; echo "=== $* (limit ${t}s)"; timeout -k 10 "$t" "$@"; local rc=$?; echo "=== rc=$rc"; return $rc; }
step 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
step 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
step 900 python bench.py --steps ${STEPS:-5} --warmup 2 > gpurun_out/bench_7b.log 2>&1 || exit 1
echo "chain ok"
