#!/bin/bash
# Round-3 batch e: the whole GPU suite at HEAD, the edge kernels alone, two plain bench runs.
# Usage: bash tools/gpu_r3e.sh
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_r3e.txt 2>&1 || { tail -40 $O/t_r3e.txt; exit 1; }
tail -2 $O/t_r3e.txt
timeout -k 10 120 python -u tools/edge_micro.py --only first_valu,first_rc,net_end,final_reduce,final_apply,in_apply > $O/edge_r3f.txt 2>&1 || { tail -20 $O/edge_r3f.txt; exit 1; }
cat $O/edge_r3f.txt
for i in 1 2; do
  timeout -k 10 150 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 20 > $O/b_r3e_$i.txt 2> $O/b_r3e_$i.err || exit 1
  echo "bench $i $(python3 -c "import json;d=json.loads(open('$O/b_r3e_$i.txt').read().splitlines()[-1]);print(d['ms_per_step'], d['value'])")"
done
echo done
