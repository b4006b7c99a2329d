#!/bin/bash
# Per-layer and per-kernel view of the training step at HEAD (GPU box):
#   layer_profile (HIP events per conv launch), a rocprofv3 kernel trace of a short bench,
#   conv_micro timings of the dominant shapes in the default arithmetic.
# Usage: bash tools/prof_layers.sh TAG
T=${1:-x}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
timeout -k 10 120 python3 $R/tools/layer_profile.py > $R/gpurun_out/layers_$T.txt 2>&1 && \
timeout -k 10 200 python3 $R/tools/conv_micro.py --pieces 16 --warm 0.5 > $R/gpurun_out/micro_$T.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tr_$T -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --c4-batches 0 --c5-steps 0 --strict-fp32-steps 0 --no-probe > $R/gpurun_out/tr_$T.json 2> $R/gpurun_out/tr_$T.log
echo rc=$?
