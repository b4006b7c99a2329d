#!/bin/bash
# PMC passes over tools/edge_micro.py cases (wave-state counters, instruction mix).
#   bash tools/pmc_edge.sh TAG "case1,case2"      (EBSDVAE_LIB selects a variant library)
T=$1; CASES=$2
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
A="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"
B="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS"
for pass in A B; do
  eval C=\$$pass
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmce_${T}_$pass -o run -- python3 $R/tools/edge_micro.py --only $CASES > $R/gpurun_out/pmce_${T}_$pass.log 2>&1 || { echo "pass $pass failed"; tail -5 $R/gpurun_out/pmce_${T}_$pass.log; exit 1; }
  python3 $R/tools/pmc_kernels.py $R/gpurun_out/pmce_${T}_$pass > $R/gpurun_out/pmce_${T}_$pass.txt
done
echo ok
