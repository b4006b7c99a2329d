#!/bin/bash
# Kernel-attached fork A/B: the whole GPU suite, step traces with EBSDVAE_KFORK=1 / 0 (idle
# between launches), then 3 bench pairs.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_p.txt 2>&1 || { tail -40 $O/t_p.txt; exit 1; }
tail -1 $O/t_p.txt
cd /tmp
for K in 1 0; do
  EBSDVAE_KFORK=$K timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tab_p_$K -o run -- python3 $R/bench.py --steps 8 --warmup 3 --no-probe --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 > $O/tab_p_$K.txt 2>&1 || exit 1
  echo "== KFORK=$K"; python3 $R/tools/step_gaps.py $O/tab_p_$K 4 5 | tail -8
done
cd $R
for i in 1 2 3; do
  for K in 1 0; do
    EBSDVAE_KFORK=$K timeout -k 10 150 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 20 > $O/b_p_${K}_$i.txt 2> $O/b_p_${K}_$i.err || exit 1
    echo "bench KFORK=$K $i $(python3 -c "import json;d=json.loads(open('$O/b_p_${K}_$i.txt').read().splitlines()[-1]);print(d['ms_per_step'], d['value'])")"
  done
done
