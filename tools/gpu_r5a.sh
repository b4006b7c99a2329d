#!/bin/bash
# Round-5 first check: determinism test, -m gpu suite, plain bench line.
# Stops at the first timeout / abort / segfault (rc >= 124); a test failure (rc 1) continues.
cd $GRAFT_REPO_ROOT
O=gpurun_out
guard() { local rc=$1; if [ $rc -ge 124 ]; then echo "stop: rc $rc"; exit $rc; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_determinism.py -v -s --timeout 120 --timeout-method thread > $O/r5_det.txt 2>&1; rc=$?; echo "det rc $rc"; guard $rc
grep -E "repeats|passed|failed" $O/r5_det.txt | tail -8
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/r5_t1.txt 2>&1; rc=$?; echo "suite rc $rc"; guard $rc; tail -3 $O/r5_t1.txt
timeout -k 10 200 python -u bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 20 > $O/r5_b1.txt 2>$O/r5_b1.err; rc=$?; echo "bench rc $rc"; guard $rc; tail -c 400 $O/r5_b1.txt
