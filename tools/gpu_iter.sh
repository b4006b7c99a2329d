#!/bin/bash
# GPU-box iteration: gpu tests, then a rocprofv3-traced short bench (no c4, no CPU baseline)
# and its per-kernel summary.  Usage: bash tools/gpu_iter.sh TAG
T=${1:-it}
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$T.txt 2>&1 || { tail -30 gpurun_out/t_$T.txt; exit 1; }
tail -1 gpurun_out/t_$T.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr_$T -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --c4-batches 0 --c5-steps 0 $BENCH_FLAGS > gpurun_out/b_$T.txt 2> gpurun_out/b_$T.err || { tail -30 gpurun_out/b_$T.err; exit 1; }
tail -1 gpurun_out/b_$T.txt | cut -c1-220
python3 tools/kernel_table.py gpurun_out/tr_$T 13
