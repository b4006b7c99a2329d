#!/bin/bash
# Round-3 batch d: the fused network end (ebsdvae_net_end) -- parity and step A/B against
# EBSDVAE_NET_END=0.  Usage: bash tools/gpu_r3d.sh
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -s -k "network_end or final or cout1 or loss" --timeout 200 --timeout-method thread > $O/t_r3d.txt 2>&1 || { tail -40 $O/t_r3d.txt; exit 1; }
grep "net_end:" $O/t_r3d.txt; tail -1 $O/t_r3d.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_fullsize.py -x -q -s --timeout 200 --timeout-method thread > $O/t_r3d2.txt 2>&1 || { tail -40 $O/t_r3d2.txt; exit 1; }
grep "fused vs\|worst weight" $O/t_r3d2.txt | head -20; tail -1 $O/t_r3d2.txt
for i in 1 2; do for v in 0 1; do
  EBSDVAE_NET_END=$v timeout -k 10 150 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 20 > $O/abne_${v}_$i.txt 2> $O/abne_${v}_$i.err || exit 1
  echo "net_end=$v $i $(python3 -c "import json;d=json.loads(open('$O/abne_${v}_$i.txt').read().splitlines()[-1]);print(d['ms_per_step'], d['value'], d['loss'])")"
done; done
echo done
