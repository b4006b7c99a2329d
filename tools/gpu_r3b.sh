#!/bin/bash
# Round-3 batch: parity of the changed kernels, bound probes of the conv / weight-gradient
# kernels, edge-kernel timings and a same-box step A/B against the HEAD-built baseline
# (lib/libebsdvae_r3base.so).  Usage: bash tools/gpu_r3b.sh
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_trainer.py -x -q --timeout 200 --timeout-method thread > $O/t_r3b.txt 2>&1 || { tail -30 $O/t_r3b.txt; exit 1; }
tail -1 $O/t_r3b.txt
bash tools/micro_variants.sh wg "wgrad32,wgrad32u,wgrad64,wgrad128,wgrad64to128,wgrad128s16" "r3base wgnomfma wgnostage" 16 || exit 1
bash tools/micro_variants.sh cv "fwd32,fwd64,fwd128,dgrad32,dgrad64,dgrad128,fwd32to64p,dgrad32to64i" "cvnomfma cvnostage" 16 || exit 1
for L in r3base new; do
  if [ $L = new ]; then LIB=$R/ebsd-vae_amd/lib/libebsdvae.so; else LIB=$R/ebsd-vae_amd/lib/libebsdvae_$L.so; fi
  echo "== $L" >> $O/edge_r3b.txt
  EBSDVAE_LIB=$LIB timeout -k 10 120 python3 tools/edge_micro.py >> $O/edge_r3b.txt 2>&1 || exit 1
done
for i in 1 2; do for L in r3base new; do
  if [ $L = new ]; then LIB=$R/ebsd-vae_amd/lib/libebsdvae.so; else LIB=$R/ebsd-vae_amd/lib/libebsdvae_$L.so; fi
  EBSDVAE_LIB=$LIB timeout -k 10 150 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 20 > $O/ab_${L}_$i.txt 2> $O/ab_${L}_$i.err || exit 1
  echo "$L $i $(python3 -c "import json;d=json.loads(open('$O/ab_${L}_$i.txt').read().splitlines()[-1]);print(d['ms_per_step'], d['value'], d['kernel_families_ms_per_step'])")"
done; done
timeout -k 10 120 python3 tools/layer_profile.py --serial > $O/layers_serial.txt 2>&1 || exit 1
echo done
