#!/bin/bash
# Round-3 batch c: the 32x32x16 weight-gradient kernel -- parity, alone (vs EBSDVAE_WG_MF32=0)
# and in the step.  Usage: bash tools/gpu_r3c.sh
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "wgrad" --timeout 200 --timeout-method thread > $O/t_r3c.txt 2>&1 || { tail -40 $O/t_r3c.txt; exit 1; }
tail -1 $O/t_r3c.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > $O/t_r3c2.txt 2>&1 || { tail -40 $O/t_r3c2.txt; exit 1; }
tail -1 $O/t_r3c2.txt
for v in 0 1; do echo "== mf32=$v" >> $O/mv_wg32.txt; EBSDVAE_WG_MF32=$v timeout -k 10 200 python3 tools/conv_micro.py --pieces 16 --warm 0.5 --only wgrad32,wgrad32u,wgrad64,wgrad128,wgrad64to128,wgrad128s16 >> $O/mv_wg32.txt 2>&1 || exit 1; done
cat $O/mv_wg32.txt | grep -v amdgpu.ids
for i in 1 2; do for v in 0 1; do
  EBSDVAE_WG_MF32=$v timeout -k 10 150 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 20 > $O/ab32_${v}_$i.txt 2> $O/ab32_${v}_$i.err || exit 1
  echo "mf32=$v $i $(python3 -c "import json;d=json.loads(open('$O/ab32_${v}_$i.txt').read().splitlines()[-1]);print(d['ms_per_step'], d['value'], d['kernel_families_ms_per_step'])")"
done; done
echo done
