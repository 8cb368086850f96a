#!/bin/bash
# 7B bench step under rocprofv3 with kernel + roctx marker tracing: per-kernel stats and the ZeRO phase ranges
# (fetch / all-gather issue / reduce / optimizer step, from utils/nvtx.instrument_w_nvtx). No PMC counters here.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats -d gpurun_out/prof_markers -o run \
  --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof_markers.log 2>&1
echo "rc=$?"
