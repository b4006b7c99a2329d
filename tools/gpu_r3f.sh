#!/bin/bash
# Round-3 batch f: serial per-layer profile, conv_micro of every case, and a kernel trace of
# unprobed (overlapped) steps.  Usage: bash tools/gpu_r3f.sh
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd $R
timeout -k 10 120 python3 tools/layer_profile.py --serial > $O/layers_r3f.txt 2>&1 || { tail $O/layers_r3f.txt; exit 1; }
timeout -k 10 300 python3 tools/conv_micro.py --pieces 16 --warm 0.5 > $O/micro_r3f.txt 2>&1 || { tail $O/micro_r3f.txt; exit 1; }
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_r3f -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --no-probe > $O/tr_r3f.json 2> $O/tr_r3f.log || exit 1
echo done
