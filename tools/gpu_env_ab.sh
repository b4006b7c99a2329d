#!/bin/bash
# Same-box A/B of an engine switch: bench lines alternating VAR=A / VAR=B.
# Usage: bash tools/gpu_env_ab.sh TAG VAR A B [pairs]
T=$1; V=$2; A=$3; B=$4; NP=${5:-2}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd $R
for i in $(seq 1 $NP); do
  for X in $A $B; do
    env $V=$X timeout -k 10 150 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 20 > $O/ab_${T}_${X}_$i.txt 2> $O/ab_${T}_${X}_$i.err || { tail -20 $O/ab_${T}_${X}_$i.err; exit 1; }
    echo "$V=$X $i $(python3 -c "import json;d=json.loads(open('$O/ab_${T}_${X}_$i.txt').read().splitlines()[-1]);print(d['ms_per_step'], d['value'])")"
  done
done
