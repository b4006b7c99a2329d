#!/bin/bash
# PMC passes over conv_micro cases in the default (f16x3) arithmetic.
#   bash tools/pmc_conv.sh TAG "case1,case2" [pieces]
# pass A: MFMA-busy / wave-state counters; pass B: instruction mix and LDS bank conflicts.
T=$1; CASES=$2; P=${3:-16}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
A="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
B="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM"
for pass in A B; do
  eval C=\$$pass
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc_${T}_$pass -o run -- python3 $R/tools/conv_micro.py --only $CASES --pieces $P --reps 5 --warm 0.3 > $R/gpurun_out/pmc_${T}_$pass.log 2>&1 || { echo "pass $pass failed"; tail -5 $R/gpurun_out/pmc_${T}_$pass.log; exit 1; }
  python3 $R/tools/pmc_kernels.py $R/gpurun_out/pmc_${T}_$pass > $R/gpurun_out/pmc_${T}_$pass.txt
done
echo ok
