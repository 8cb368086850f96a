#!/bin/bash
# Kernel-level profile of BLOOM-176B-shaped decode (${L:-8} layers, batch ${B:-1}, ${Q:-4}-bit weights, no graph)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bloom -o run --output-format csv -- python3 tools/bench_bloom176b_int8.py --layers ${L:-8} --batches ${B:-1} --gen ${GEN:-32} --graph 0 --bits ${Q:-4} --group ${GS:-128} > gpurun_out/prof_bloom.log 2>&1 || { tail -20 gpurun_out/prof_bloom.log; exit 1; }
tail -2 gpurun_out/prof_bloom.log
python tools/kstats.py gpurun_out/prof_bloom/run_kernel_stats.csv 22 || head -30 gpurun_out/prof_bloom/run_kernel_stats.csv
find gpurun_out/prof_bloom -name "*_trace.csv" -size +20M -delete
echo "chain ok"
