#!/bin/bash
# Kernel traces of the plain training step (no probe, no side legs) for env A/B runs.
# Usage: bash tools/trace_ab.sh TAG [VAR=VALUE ...]
T=$1; shift
export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tab_$T -o run -- \
  python3 bench.py --steps 8 --warmup 3 --no-probe --no-cpu-baseline --strict-fp32-steps 0 \
  --c4-batches 0 --c5-steps 0 > gpurun_out/tab_$T.txt 2>&1
