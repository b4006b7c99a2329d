#!/bin/bash
# Round-3 bound probe: conv / weight-gradient kernels alone with their MFMAs or their staging
# compiled out (timing variants, wrong results), a serial per-layer profile and a serial
# kernel trace of the step.  Usage: bash tools/gpu_r3_probe.sh
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
bash $R/tools/micro_variants.sh wg "wgrad32,wgrad32u,wgrad64,wgrad128,wgrad64to128,wgrad128s16" "wgnomfma wgnostage" 16 || exit 1
bash $R/tools/micro_variants.sh cv "fwd32,fwd64,fwd128,dgrad32,dgrad64,dgrad128,fwd32to64p,dgrad32to64i" "cvnomfma cvnostage" 16 || exit 1
timeout -k 10 120 python3 $R/tools/layer_profile.py --serial > $O/layers_serial.txt 2>&1 || exit 1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_serial -o run -- python3 $R/bench.py --steps 6 --warmup 2 --probe-every 1 --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 > $O/b_serial.txt 2> $O/b_serial.err || exit 1
echo done
