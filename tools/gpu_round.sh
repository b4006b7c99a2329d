#!/bin/bash
# Round-end GPU pass: full gpu test suite, smoke(), then tools/prof_round.sh (rocprofv3 trace,
# PMC FETCH/WRITE passes, plain bench).  Usage: bash tools/gpu_round.sh
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_round.txt 2>&1 || { tail -40 gpurun_out/t_round.txt; exit 1; }
tail -1 gpurun_out/t_round.txt
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { tail -20 gpurun_out/smoke.txt; exit 1; }
tail -1 gpurun_out/smoke.txt
bash tools/prof_round.sh
