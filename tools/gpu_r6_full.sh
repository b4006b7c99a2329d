# round 6: the whole GPU suite, smoke and the default bench line at HEAD
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r6_full_tests.txt 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6_full_tests.txt; exit 1; }
tail -3 gpurun_out/r6_full_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_smoke.txt 2>&1 || { echo SMOKE_FAILED; exit 1; }
timeout -k 10 900 python bench.py > gpurun_out/r6_bench.json 2> gpurun_out/r6_bench.err
