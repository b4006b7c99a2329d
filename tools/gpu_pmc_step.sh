#!/bin/bash
# Per-kernel HBM bytes of the bench step (serial streams): separate FETCH_SIZE / WRITE_SIZE
# passes over 1 + 3 steps, summarised per kernel (tools/pmc_kernels.py).
# Usage: bash tools/gpu_pmc_step.sh TAG [bench args...]
T=$1; shift
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  EBSDVAE_WGRAD_STREAM=0 timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d $O/pmcs_${T}_$C -o run -- python3 $R/bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --no-probe --steps 3 --warmup 1 "$@" > $O/pmcs_${T}_$C.log 2>&1 || { echo "pass $C failed"; tail -5 $O/pmcs_${T}_$C.log; exit 1; }
  python3 $R/tools/pmc_kernels.py $O/pmcs_${T}_$C > $O/pmcs_${T}_$C.txt
done
head -30 $O/pmcs_${T}_FETCH_SIZE.txt | cut -c1-160
