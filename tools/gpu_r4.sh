#!/bin/bash
# Round-4 GPU probe: default bench line (no CPU baseline / c4 / c5 / strict), per-layer
# serial profile, and a rocprofv3 kernel trace of the plain step.
# Usage: bash tools/gpu_r4.sh TAG [trace:0|1]
T=${1:-r4}; TR=${2:-1}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd $R
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 20 > $O/b_${T}_$i.txt 2> $O/b_${T}_$i.err || { tail -20 $O/b_${T}_$i.err; exit 1; }
  echo "bench $i $(python3 -c "import json;d=json.loads(open('$O/b_${T}_$i.txt').read().splitlines()[-1]);print(d['ms_per_step'], d['value'], d['roofline']['frac'])")"
done
timeout -k 10 200 python3 tools/layer_profile.py --serial > $O/layers_$T.txt 2>&1 || { tail -20 $O/layers_$T.txt; exit 1; }
tail -5 $O/layers_$T.txt
if [ "$TR" = 1 ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$T -o run -- python3 $R/bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 20 --no-probe > $O/prof_$T.log 2>&1 || { tail -20 $O/prof_$T.log; exit 1; }
  cd $R
fi
echo done
