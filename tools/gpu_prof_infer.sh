#!/bin/bash
# Kernel-level profile of Llama-2-7B decode (batch ${B:-1}) -> gpurun_out/prof_infer/
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_infer -o run --output-format csv -- python3 tools/bench_infer.py --batches ${B:-1} --prompt 512 --gen 32 --graph 0 > gpurun_out/prof_infer.log 2>&1
echo "rc=$?"
