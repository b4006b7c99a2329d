#!/bin/bash
# Serial-stream kernel trace of the default bench step (weight gradients on the main stream,
# so every kernel's duration is its own): rocprofv3 CSV stats + the trace database summary.
# Usage: bash tools/gpu_serial.sh TAG
T=${1:-ser}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd /tmp
EBSDVAE_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$T -o run -- python3 $R/bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 20 --no-probe > $O/prof_$T.log 2>&1 || { tail -20 $O/prof_$T.log; exit 1; }
cd $R
python3 tools/trace_db.py $(ls $O/prof_$T/*.db $O/prof_$T/*/*.db 2>/dev/null | head -1) --steps 10 > $O/trace_$T.txt 2>&1
head -16 $O/trace_$T.txt
