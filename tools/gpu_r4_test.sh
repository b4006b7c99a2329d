#!/bin/bash
# Round-4 GPU check: kernel parity tests of the fused / staged input gradients, the trainer and
# full-size gates, then the bench probe (tools/gpu_r4.sh).
# Usage: bash tools/gpu_r4_test.sh TAG [pytest -k expr]
T=${1:-r4t}; K=${2:-"dgrad or staged or instance_norm or fused or first"}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "$K" > $O/tk_$T.txt 2>&1 || { tail -40 $O/tk_$T.txt; exit 1; }
tail -2 $O/tk_$T.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_fullsize.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > $O/tt_$T.txt 2>&1 || { tail -40 $O/tt_$T.txt; exit 1; }
tail -2 $O/tt_$T.txt
bash tools/gpu_r4.sh $T 0
