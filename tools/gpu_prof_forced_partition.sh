#!/bin/bash
# 7B ZeRO-3 step on ONE GPU through the full multi-rank code path (DS_ZERO_FORCE_PARTITION=1: partitioned groups,
# all-gather on the prefetch stream, reduce-scatter on the reduction stream, RCCL kernels) under rocprofv3 kernel +
# roctx marker tracing; then tools/comm_overlap.py quantifies exposed communication. Timed window starts at the
# 4th flash-attention forward of the last step (steps 1-2 are warmup) -> conservative.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp DS_ZERO_FORCE_PARTITION=1
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/forced_bench.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats -d gpurun_out/prof_forced -o run \
  --output-format csv -- python3 bench.py --steps 1 --warmup 2 > gpurun_out/prof_forced.log 2>&1 || exit 1
echo "prof ok"
