#!/bin/bash
# A/B of the in-tree library against ebsd-vae_amd/lib/libebsdvae_old.so (the previous commit,
# built in a worktree): parity tests (-k expr), per-layer serial profiles of both, then bench
# pairs alternating new / old.
# Usage: bash tools/gpu_ab2.sh TAG "pytest -k expr" [pairs]
T=${1:-ab}; K=${2:-"conv or split or fused or pooled"}; NP=${3:-2}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd $R
NEW=$R/ebsd-vae_amd/lib/libebsdvae.so; OLD=$R/ebsd-vae_amd/lib/libebsdvae_old.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "$K" > $O/tk_$T.txt 2>&1 || { tail -40 $O/tk_$T.txt; exit 1; }
tail -1 $O/tk_$T.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/tt_$T.txt 2>&1 || { tail -40 $O/tt_$T.txt; exit 1; }
tail -1 $O/tt_$T.txt
for L in new old; do
  if [ $L = new ]; then LIB=$NEW; else LIB=$OLD; fi
  EBSDVAE_LIB=$LIB timeout -k 10 200 python3 tools/layer_profile.py --serial > $O/lay_${T}_$L.txt 2>&1 || { tail -20 $O/lay_${T}_$L.txt; exit 1; }
done
python3 tools/layer_diff.py $O/lay_${T}_old.txt $O/lay_${T}_new.txt
for i in $(seq 1 $NP); do
  for L in new old; do
    if [ $L = new ]; then LIB=$NEW; else LIB=$OLD; fi
    EBSDVAE_LIB=$LIB timeout -k 10 150 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 20 > $O/b_${T}_${L}_$i.txt 2> $O/b_${T}_${L}_$i.err || { tail -20 $O/b_${T}_${L}_$i.err; exit 1; }
    echo "bench $L $i $(python3 -c "import json;d=json.loads(open('$O/b_${T}_${L}_$i.txt').read().splitlines()[-1]);print(d['ms_per_step'], d['value'])")"
  done
done
