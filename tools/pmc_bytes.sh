#!/bin/bash
# HBM byte counters over conv_micro cases, one PMC pass per counter (FETCH_SIZE, WRITE_SIZE):
#   bash tools/pmc_bytes.sh TAG "case1,case2" [pieces]
T=$1; CASES=$2; P=${3:-16}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmcb_${T}_$C -o run -- python3 $R/tools/conv_micro.py --only $CASES --pieces $P --reps 5 --warm 0.3 > $R/gpurun_out/pmcb_${T}_$C.log 2>&1 || { echo "pass $C failed"; tail -5 $R/gpurun_out/pmcb_${T}_$C.log; exit 1; }
  python3 $R/tools/pmc_kernels.py $R/gpurun_out/pmcb_${T}_$C > $R/gpurun_out/pmcb_${T}_$C.txt
done
echo ok
