#!/bin/bash
# Round-3 batch g: does the Infinity Cache (256 MiB) serve a layer whose tensors fit in it?
# conv_micro / edge_micro of the memory-heavy shapes at B = 32, 64, 128, 256 (time per image).
# Usage: bash tools/gpu_r3g.sh
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd $R
: > $O/l3_r3g.txt
for b in 32 64 128 256; do
  echo "== B=$b" >> $O/l3_r3g.txt
  timeout -k 10 200 python3 tools/conv_micro.py --pieces 16 --warm 0.3 --batch $b --only fwd32,dgrad32,wgrad32,fwd64,dgrad64,wgrad64 >> $O/l3_r3g.txt 2>&1 || exit 1
  timeout -k 10 100 python3 tools/edge_micro.py --batch $b --only in_apply,final_apply,net_end >> $O/l3_r3g.txt 2>&1 || exit 1
done
echo done
