#!/bin/bash
# Kernel trace of one bench configuration (serial streams unless SIDE=1), summarised per
# iteration.  Usage: bash tools/gpu_trace.sh TAG MARKER STEPS "bench args..."
T=$1; MK=${2:-adam_kernel}; NS=${3:-10}; shift 3
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd /tmp
if [ "${SIDE:-0}" = 1 ]; then unset EBSDVAE_WGRAD_STREAM; else export EBSDVAE_WGRAD_STREAM=0; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$T -o run -- python3 $R/bench.py --no-cpu-baseline --strict-fp32-steps 0 --no-probe "$@" > $O/prof_$T.log 2>&1 || { tail -20 $O/prof_$T.log; exit 1; }
cd $R
python3 tools/trace_db.py $(ls $O/prof_$T/*.db $O/prof_$T/*/*.db 2>/dev/null | head -1) --steps $NS --marker $MK > $O/trace_$T.txt 2>&1
head -20 $O/trace_$T.txt
