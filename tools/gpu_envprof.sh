#!/bin/bash
# A/B of a library env switch: parity tests with VAR=B, serial per-layer profiles of A and B,
# then bench pairs.  Usage: bash tools/gpu_envprof.sh TAG VAR A B "pytest -k expr" [pairs]
T=$1; V=$2; A=$3; B=$4; K=${5:-"vae128"}; NP=${6:-2}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd $R
env $V=$B timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_fullsize.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "$K" > $O/tk_$T.txt 2>&1 || { tail -40 $O/tk_$T.txt; exit 1; }
tail -1 $O/tk_$T.txt
for X in $A $B; do
  env $V=$X timeout -k 10 200 python3 tools/layer_profile.py --serial > $O/lay_${T}_$X.txt 2>&1 || { tail -20 $O/lay_${T}_$X.txt; exit 1; }
done
python3 tools/layer_diff.py $O/lay_${T}_$A.txt $O/lay_${T}_$B.txt | head -30
bash tools/gpu_env_ab.sh $T $V $A $B $NP
