#!/bin/bash
# Two rocprofv3 counter passes over tools/run_flash_bwd_once.py (each pass <= 8 SQ counters), summaries to gpurun_out/
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS -d $R/gpurun_out/pmc/p1 -o p1 --output-format csv -- python3 $R/tools/run_flash_bwd_once.py > $R/gpurun_out/pmc/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $R/gpurun_out/pmc/p2 -o p2 --output-format csv -- python3 $R/tools/run_flash_bwd_once.py > $R/gpurun_out/pmc/p2.log 2>&1
echo pmc-done
