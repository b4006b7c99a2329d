#!/bin/bash
# c4 (encoder inference) A/B of the in-tree library with and without the pooled producers' full-resolution output (EBSDVAE_EVAL_Y): the full
# -m gpu suite, then the bench's c4 leg alternating new / old.
# Usage: bash tools/gpu_c4.sh TAG [pairs]
T=${1:-c4}; NP=${2:-2}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd $R
LIB=$R/ebsd-vae_amd/lib/libebsdvae.so
[ "${SKIPT:-0}" = 1 ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_$T.txt 2>&1 || { tail -30 $O/t_$T.txt; exit 1; }
[ "${SKIPT:-0}" = 1 ] || tail -1 $O/t_$T.txt
for i in $(seq 1 $NP); do
  for L in new old; do
    if [ $L = new ]; then EY=0; else EY=1; fi
    EBSDVAE_EVAL_Y=$EY timeout -k 10 200 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c5-steps 0 --steps 10 > $O/b_${T}_${L}_$i.txt 2> $O/b_${T}_${L}_$i.err || exit 1
    echo "bench $L $i $(python3 -c "
import json;d=json.loads(open('$O/b_${T}_${L}_$i.txt').read().splitlines()[-1]);c=d['c4_encoder_latents']
print(d['ms_per_step'], c['ms_per_batch'], c['value'], c['engine_only']['value'])")"
  done
done
echo done
