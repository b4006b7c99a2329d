#!/bin/bash
# GPU check of a change: the named test files (verbose, prints kept), then optionally the
# serial kernel trace (tools/gpu_serial.sh).  Usage: bash tools/gpu_check.sh TAG "tests..." [serial:0|1]
T=${1:-chk}; TESTS=${2:-tests}; SER=${3:-0}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest $TESTS -x -v -s -m gpu --timeout 300 --timeout-method thread > $O/t_$T.txt 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|residue|worst" $O/t_$T.txt | tail -80
[ $rc = 0 ] || { tail -40 $O/t_$T.txt; exit 1; }
if [ "$SER" = 1 ]; then bash tools/gpu_serial.sh $T || exit 1; fi
echo done
