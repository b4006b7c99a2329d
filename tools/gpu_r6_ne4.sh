# round 6: net_end variants (six-step unroll, branch-free g1 ring) micro A/B; fork-event scope bench A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2; do for L in default neu2 nebr; do
  if [ $L = default ]; then unset EBSDVAE_LIB; else export EBSDVAE_LIB=ebsd-vae_amd/lib/libebsdvae_$L.so; fi
  timeout -k 10 120 python3 tools/edge_micro.py --only net_end 2>&1 | grep -v amdgpu.ids | sed "s/^/$L /" || exit 1
done; done
unset EBSDVAE_LIB
for i in 1 2; do for S in 0 1; do
  EBSDVAE_FORK_DEVICE_SCOPE=$S timeout -k 10 200 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 30 > gpurun_out/fs_$S.txt 2>/dev/null || exit 1
  echo "device_scope=$S bench $(python3 -c "import json;d=json.loads(open('gpurun_out/fs_$S.txt').read().splitlines()[-1]);print(d['ms_per_step'])")"
done; done
