#!/bin/bash
# Knob sweep on the current default step (two runs each, same box).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
for i in 1 2; do
  for cfg in "X=0" "EBSDVAE_WG_BLOCKS=768" "EBSDVAE_WG_BLOCKS=1024" "HIP_FORCE_DEV_KERNARG=1" "EBSDVAE_WRES=0" "EBSDVAE_CONV_SMALL1=0" "EBSDVAE_KFORK=0"; do
    env $cfg timeout -k 10 150 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 20 > $O/s.txt 2> $O/s.err || { tail $O/s.err; exit 1; }
    echo "$cfg run $i: $(python3 -c "import json;d=json.loads(open('$O/s.txt').read().splitlines()[-1]);print(d['ms_per_step'], d['value'])")"
  done
done
