#!/bin/bash
# rocprofv3 kernel-stats profile of a short 7B bench run (2 timed steps + 1 warmup); summary CSV -> gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
DS_BENCH_FORCED=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof7b" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 2 --warmup 1 ${BENCH_ARGS} > "$R/gpurun_out/prof7b.log" 2>&1 || { tail -20 "$R/gpurun_out/prof7b.log"; exit 1; }
cd "$R"
f=$(find gpurun_out/prof7b -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/prof7b_kernel_stats.csv
head -25 gpurun_out/prof7b_kernel_stats.csv | cut -c1-200
find gpurun_out/prof7b -name "*_trace.csv" -delete
tail -1 gpurun_out/prof7b.log | cut -c1-300
