#!/bin/bash
# rocprofv3 kernel trace + counter passes over tools/run_i8_once.py (int8 MFMA skinny GEMM), to gpurun_out/pmc_i8
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_i8
rm -rf $O; mkdir -p $O
for c in 0 1; do
  DS_I8_CFG=$c timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/kt$c -o kt --output-format csv -- python3 $R/tools/run_i8_once.py > $O/kt$c.log 2>&1
done
DS_I8_CFG=1 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_WAVES SQ_INSTS_SALU -d $O/p1 -o p1 --output-format csv -- python3 $R/tools/run_i8_once.py > $O/p1.log 2>&1
DS_I8_CFG=1 timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE TCC_EA0_RDREQ_sum -d $O/p3 -o p3 --output-format csv -- python3 $R/tools/run_i8_once.py > $O/p3.log 2>&1
echo pmc-done
