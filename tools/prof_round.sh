export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r01_trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --c4-batches 0 --c5-steps 0 > $R/gpurun_out/r01_bench_traced.json 2> $R/gpurun_out/r01_trace.log && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r01_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe --c4-batches 0 --c5-steps 0 > $R/gpurun_out/r01_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/r01_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe --c4-batches 0 --c5-steps 0 > $R/gpurun_out/r01_write.log 2>&1 && \
python3 $R/tools/pmc_traffic.py --trace $R/gpurun_out/r01_trace --fetch $R/gpurun_out/r01_fetch --write $R/gpurun_out/r01_write --steps 25 --out $R/gpurun_out/pmc_traffic.json > /dev/null && \
cp $R/gpurun_out/pmc_traffic.json $R/profiles/pmc_traffic.json && \
timeout -k 10 300 python3 $R/bench.py > $R/gpurun_out/r01_bench.json 2> $R/gpurun_out/r01_bench.err
rc=$?
cp $R/gpurun_out/r01_trace/run_kernel_stats.csv $R/profiles/r01_kernel_stats.csv
cp $R/gpurun_out/r01_bench_traced.json $R/gpurun_out/r01_bench.json $R/profiles/
echo rc=$rc
cat $R/gpurun_out/r01_bench_traced.json; cat $R/gpurun_out/r01_bench.json
