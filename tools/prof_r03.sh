#!/bin/bash
# Round-3 evidence at HEAD: the round-2 recipe (tools/prof_r02.sh r03: kernel trace, FETCH /
# WRITE passes, step and kernel PMC passes, the default bench line) plus the serial per-layer
# profile and a trace of unprobed (overlapped) steps for the stream timeline.
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd /tmp
bash $R/tools/prof_r02.sh r03 || exit 1
timeout -k 10 120 python3 $R/tools/layer_profile.py --serial > $O/r03_layers.txt 2>&1 || exit 1
cp $O/r03_layers.txt $R/profiles/
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03_overlap -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --no-probe > $O/r03_overlap.json 2> $O/r03_overlap.log || exit 1
cp $O/r03_overlap/run_kernel_stats.csv $R/profiles/r03_overlap_kernel_stats.csv
echo prof done
