#!/bin/bash
# Round-2 evidence at HEAD (GPU box), everything under gpurun_out/, summaries copied to profiles/:
#   1. rocprofv3 --kernel-trace --stats of bench.py (probe on: its JSON line and the trace
#      time the same launches; 5 warm-up + 20 timed steps);
#   2. separate FETCH_SIZE and WRITE_SIZE passes over a 1+3-step bench -> pmc_traffic.json
#      (per-family bytes per launch and per step; bench.py reads roofline.traffic from it);
#   3. MFMA-busy / wave-state and instruction-mix / LDS-bank-conflict passes over the
#      conv_micro cases of the f16x3 kernels (tools/pmc_conv.sh), and the MFMA-busy pass over
#      the bench step itself;
#   4. the default bench.py line (CPU baseline, c4, c5, strict fp32 rate).
T=${1:-r02}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
B="python3 $R/bench.py --probe-every 5 --no-cpu-baseline --c4-batches 0 --c5-steps 0 --strict-fp32-steps 0"
A="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_trace -o run -- $B --steps 20 --warmup 5 > $O/${T}_bench_traced.json 2> $O/${T}_trace.log && echo trace ok && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${T}_fetch -o run -- $B --steps 3 --warmup 1 --no-probe > $O/${T}_fetch.log 2>&1 && echo fetch ok && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${T}_write -o run -- $B --steps 3 --warmup 1 --no-probe > $O/${T}_write.log 2>&1 && echo write ok && \
python3 $R/tools/pmc_traffic.py --trace $O/${T}_trace --fetch $O/${T}_fetch --write $O/${T}_write --steps 25 --probed 5:20:5 --out $O/pmc_traffic.json > /dev/null && \
cp $O/pmc_traffic.json $R/profiles/pmc_traffic.json && cp $O/pmc_traffic.json $R/profiles/${T}_pmc_traffic.json && \
timeout -s KILL 200 rocprofv3 --pmc $A --output-format csv -d $O/${T}_pmc_step -o run -- $B --steps 3 --warmup 1 --no-probe > $O/${T}_pmc_step.log 2>&1 && echo step pmc ok && \
python3 $R/tools/pmc_kernels.py $O/${T}_pmc_step > $O/${T}_pmc_step.txt && \
bash $R/tools/pmc_conv.sh ${T}c "fwd32,fwd64,fwd128,dgrad32,dgrad64,dgrad128,wgrad32,wgrad64,wgrad128" && \
timeout -k 10 600 python3 $R/bench.py > $O/${T}_bench.json 2> $O/${T}_bench.err
rc=$?
cp $O/${T}_trace/run_kernel_stats.csv $R/profiles/${T}_kernel_stats.csv 2>/dev/null
cp $O/${T}_bench_traced.json $O/${T}_bench.json $O/${T}_pmc_step.txt $R/profiles/ 2>/dev/null
cp $O/pmc_${T}c_A.txt $R/profiles/${T}_pmc_conv_mfma.txt 2>/dev/null
cp $O/pmc_${T}c_B.txt $R/profiles/${T}_pmc_conv_lds.txt 2>/dev/null
echo rc=$rc
