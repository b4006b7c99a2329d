# round 6: weight-gradient slice count (EBSDVAE_WG_BLOCKS: block target per launch) -- step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2; do for V in 512 256 1024 384; do
  EBSDVAE_WG_BLOCKS=$V timeout -k 10 200 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 30 > gpurun_out/wgb_$V.txt 2>/dev/null || exit 1
  echo "blocks=$V bench $(python3 -c "import json;d=json.loads(open('gpurun_out/wgb_$V.txt').read().splitlines()[-1]);print(d['ms_per_step'], d['kernel_families_ms_per_step'])")"
done; done
