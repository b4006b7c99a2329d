#!/bin/bash
# One experiment per call (round 5): parity tests at the default settings, conv_micro cases
# and same-box bench pairs for each value of one switch.
# Usage: bash tools/gpu_exp.sh TAG "pytest args|-" "micro cases|-" VAR "v1 v2 ..." [pairs]
# Stops at the first timeout / abort / segfault (rc >= 124); a test failure (rc 1) stops too.
T=$1; TESTS=$2; MICRO=$3; VAR=$4; VALS=$5; NP=${6:-2}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
if [ "$TESTS" != "-" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -q -x --timeout 200 --timeout-method thread > $O/x_${T}_t.txt 2>&1; rc=$?
  tail -2 $O/x_${T}_t.txt; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/x_${T}_t.txt | head -20; exit $rc; }
fi
if [ "$MICRO" != "-" ]; then
  for X in $VALS; do
    echo "== $VAR=$X"
    env $VAR=$X timeout -k 10 200 python3 tools/conv_micro.py --pieces 16 --warm 0.5 --only $MICRO 2>&1 | grep -v amdgpu.ids; rc=${PIPESTATUS[0]}
    [ $rc -ne 0 ] && exit $rc
  done
fi
for i in $(seq 1 $NP); do
  for X in $VALS; do
    env $VAR=$X timeout -k 10 150 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 20 > $O/x_${T}_${X}_$i.txt 2> $O/x_${T}_${X}_$i.err; rc=$?
    [ $rc -ne 0 ] && { tail -20 $O/x_${T}_${X}_$i.err; exit $rc; }
    echo "bench $VAR=$X $i $(python3 -c "import json;d=json.loads(open('$O/x_${T}_${X}_$i.txt').read().splitlines()[-1]);print(d['ms_per_step'], d['value'], d['kernel_families_ms_per_step'])")"
  done
done
