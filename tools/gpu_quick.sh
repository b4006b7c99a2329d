#!/bin/bash
# GPU-box quick check: gpu tests, then a traced short bench.  Usage: bash tools/gpu_quick.sh TAG
T=${1:-q}
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t_$T.txt 2>&1 || { tail -30 gpurun_out/t_$T.txt; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr_$T -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_$T.txt 2> gpurun_out/b_$T.err || { tail -30 gpurun_out/b_$T.err; exit 1; }
tail -1 gpurun_out/t_$T.txt
tail -1 gpurun_out/b_$T.txt | cut -c1-160
