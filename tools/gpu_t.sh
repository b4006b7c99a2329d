#!/bin/bash
# Round-end rehearsal: smoke() and the default bench line, as the driver runs them.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_t.txt 2>&1 || { tail -20 $O/smoke_t.txt; exit 1; }
tail -3 $O/smoke_t.txt
timeout -k 10 600 python3 bench.py > $O/bench_t.json 2> $O/bench_t.err || { tail -20 $O/bench_t.err; exit 1; }
tail -1 $O/bench_t.json | cut -c1-400
