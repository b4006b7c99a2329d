#!/bin/bash
# Wide (co 128) weight-gradient blocks as the default: the whole GPU suite, then 3 bench pairs
# against EBSDVAE_WG_CO128=0.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_r.txt 2>&1 || { tail -40 $O/t_r.txt; exit 1; }
tail -1 $O/t_r.txt
for i in 1 2 3; do
  for K in 1 0; do
    EBSDVAE_WG_CO128=$K timeout -k 10 150 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 20 > $O/b_r_${K}_$i.txt 2> $O/b_r_${K}_$i.err || exit 1
    echo "bench CO128=$K $i $(python3 -c "import json;d=json.loads(open('$O/b_r_${K}_$i.txt').read().splitlines()[-1]);print(d['ms_per_step'], d['value'])")"
  done
done
