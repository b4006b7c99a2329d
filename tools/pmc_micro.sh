#!/bin/bash
# one PMC pass over a conv_micro case: bash tools/pmc_micro.sh CASE TAG "COUNTERS"
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc $3 --output-format csv -d gpurun_out/pmc_$2 -o run -- python3 tools/conv_micro.py --only $1 --reps 5 > gpurun_out/pmc_$2.log 2>&1 && python3 tools/pmc_kernels.py gpurun_out/pmc_$2 --match conv3x3
