#!/bin/bash
# Weight-gradient knob A/B on the current step: default, EBSDVAE_WG_CO128=1, WG_BLOCKS=384 / 768.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
for i in 1 2; do
  for cfg in "X=0" "EBSDVAE_WG_CO128=1" "EBSDVAE_WG_BLOCKS=384" "EBSDVAE_WG_BLOCKS=768"; do
    env $cfg timeout -k 10 150 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 20 > $O/q.txt 2> $O/q.err || { tail $O/q.err; exit 1; }
    echo "$cfg run $i: $(python3 -c "import json;d=json.loads(open('$O/q.txt').read().splitlines()[-1]);print(d['ms_per_step'], d['value'])")"
  done
done
