#!/bin/bash
# Kernel-level profile of Llama-2-7B decode (batch ${B:-1}, weight bits ${Q:-0}) -> gpurun_out/prof_infer/
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_infer -o run --output-format csv -- python3 tools/bench_infer.py --batches ${B:-1} --prompt ${PROMPT:-128} --gen ${GEN:-64} --graph ${GRAPH:-0} --quant-bits ${Q:-0} --group-size ${GS:-128} > gpurun_out/prof_infer.log 2>&1 || { tail -20 gpurun_out/prof_infer.log; exit 1; }
tail -3 gpurun_out/prof_infer.log
python tools/kstats.py gpurun_out/prof_infer/run_kernel_stats.csv 25 || head -30 gpurun_out/prof_infer/run_kernel_stats.csv
find gpurun_out/prof_infer -name "*_trace.csv" -size +20M -delete
echo "chain ok"
