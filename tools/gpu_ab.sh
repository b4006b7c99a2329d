#!/bin/bash
# A/B of the in-tree library against ebsd-vae_amd/lib/libebsdvae_old.so (the previous HEAD,
# built in a worktree): kernel parity tests, conv_micro of the dominant shapes for both
# libraries, then the bench alternating new / old.
# Usage: bash tools/gpu_ab.sh TAG [micro cases] [bench pairs]
T=${1:-ab}; C=${2:-fwd32,fwd64,fwd128,dgrad32,dgrad64,dgrad128,wgrad32,wgrad64,wgrad128}; NP=${3:-2}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd $R
NEW=$R/ebsd-vae_amd/lib/libebsdvae.so; OLD=$R/ebsd-vae_amd/lib/libebsdvae_old.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_trainer.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/t_$T.txt 2>&1 || { tail -30 $O/t_$T.txt; exit 1; }
tail -1 $O/t_$T.txt
: > $O/micro_$T.txt
for L in new old; do
  if [ $L = new ]; then LIB=$NEW; else LIB=$OLD; fi
  echo "== $L" >> $O/micro_$T.txt
  EBSDVAE_LIB=$LIB timeout -k 10 200 python3 tools/conv_micro.py --pieces 16 --warm 0.5 --only $C >> $O/micro_$T.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/micro_$T.txt
for i in $(seq 1 $NP); do
  for L in new old; do
    if [ $L = new ]; then LIB=$NEW; else LIB=$OLD; fi
    EBSDVAE_LIB=$LIB timeout -k 10 150 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 20 > $O/b_${T}_${L}_$i.txt 2> $O/b_${T}_${L}_$i.err || exit 1
    echo "bench $L $i $(python3 -c "import json;d=json.loads(open('$O/b_${T}_${L}_$i.txt').read().splitlines()[-1]);print(d['ms_per_step'], d['value'])")"
  done
done
echo done
