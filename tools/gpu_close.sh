#!/bin/bash
# Re-entry closing check at HEAD: GPU suite, smoke, default bench line.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_close.txt 2>&1 || { tail -40 $O/t_close.txt; exit 1; }
tail -1 $O/t_close.txt
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_close.txt 2>&1 || { tail -20 $O/smoke_close.txt; exit 1; }
tail -1 $O/smoke_close.txt
timeout -k 10 300 python -u bench.py > $O/bench_close.txt 2>&1 || { tail -20 $O/bench_close.txt; exit 1; }
tail -1 $O/bench_close.txt
