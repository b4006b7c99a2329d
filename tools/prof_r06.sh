#!/bin/bash
# Round-6 evidence at HEAD: the round-2 recipe (tools/prof_r02.sh r06: kernel trace, FETCH /
# WRITE passes -> pmc_traffic.json, step and conv PMC passes, the default bench line), the
# serial per-layer profile, and serial-stream traces of c2 / c5 / c4 (tools/gpu_trace.sh).
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd /tmp
bash $R/tools/prof_r02.sh r06 || exit 1
timeout -k 10 150 python3 $R/tools/layer_profile.py --serial > $O/r06_layers.txt 2>&1 || exit 1
cd $R
bash tools/gpu_trace.sh r06c2 adam_kernel 10 --steps 20 --c5-steps 0 --c4-batches 0 > /dev/null || exit 1
bash tools/gpu_trace.sh r06c5 adam_kernel 8 --image-size 256 --latent-dim 64 --batch 128 --steps 10 --warmup 3 --c5-steps 0 --c4-batches 0 > /dev/null || exit 1
bash tools/gpu_trace.sh r06c4 heads_fwd 20 --steps 2 --warmup 1 --c5-steps 0 --c4-batches 30 > /dev/null || exit 1

# keep the summaries (gpurun merges back at most 64 MiB of gpurun_out/): raw traces and counter
# dumps are deleted once summarised
mkdir -p $O/r06
cp $O/r06_trace/run_kernel_stats.csv $O/r06/r06_kernel_stats.csv 2>/dev/null
cp $O/r06_bench_traced.json $O/r06_bench.json $O/r06_pmc_step.txt $O/pmc_traffic.json $O/r06_layers.txt $O/r06/ 2>/dev/null
cp $O/pmc_r06c_A.txt $O/r06/r06_pmc_conv_mfma.txt 2>/dev/null
cp $O/pmc_r06c_B.txt $O/r06/r06_pmc_conv_lds.txt 2>/dev/null
cp $O/trace_r06c2.txt $O/r06/r06_c2_serial_trace.txt; cp $O/trace_r06c5.txt $O/r06/r06_c5_serial_trace.txt; cp $O/trace_r06c4.txt $O/r06/r06_c4_serial_trace.txt
rm -rf $O/r06_trace $O/r06_fetch $O/r06_write $O/r06_pmc_step $O/pmc_r06c_A $O/pmc_r06c_B $O/prof_r06c2 $O/prof_r06c5 $O/prof_r06c4
du -sh $O
echo prof done
