#!/bin/bash
# RCCL all-reduce kernel resources.  Usage: bash tools/gpu_rccl_probe.sh
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/prof_rccl -o run -- python3 $R/tools/rccl_probe.py > $O/rccl_probe.log 2>&1 || { tail -20 $O/rccl_probe.log; exit 1; }
cd $R
python3 tools/rccl_probe.py --db $(ls $O/prof_rccl/*.db $O/prof_rccl/*/*.db 2>/dev/null | head -1) | tee $O/rccl_kernels.txt
