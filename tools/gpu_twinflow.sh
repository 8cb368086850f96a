#!/bin/bash
# Twin-Flow / tiered offload on the GPU: the engine tests, then bench_max_params runs named by the arguments.
# usage: gpu_twinflow.sh <name> "<bench_max_params args>" [<name> "<args>" ...]   (each run time-limited)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local t=$1; shift; echo "=== $* (limit ${t}s)"; timeout -k 10 "$t" "$@"; local rc=$?; echo "=== rc=$rc"; return $rc; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  step 400 python -u -m pytest tests/unit/runtime/test_zero_gpu.py tests/unit/runtime/test_offload.py -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/twinflow_tests.log 2>&1 || { tail -30 gpurun_out/twinflow_tests.log; exit 1; }
  tail -2 gpurun_out/twinflow_tests.log
fi
while [ $# -ge 2 ]; do
  name=$1; args=$2; shift 2
  step "${RUN_LIMIT:-600}" python -u tools/bench_max_params.py $args --tag "$name" \
    > "gpurun_out/maxparams_${name}.json" 2> "gpurun_out/maxparams_${name}.log" || { tail -25 "gpurun_out/maxparams_${name}.log"; exit 1; }
  tail -4 "gpurun_out/maxparams_${name}.log"; cat "gpurun_out/maxparams_${name}.json"
  rm -rf /tmp/ds_nvme_bench
done
echo "chain ok"
