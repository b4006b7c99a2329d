# round 6: net_end 64-row vs 32-row bands, micro only
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2; do for L in default th32; do
  if [ $L = default ]; then unset EBSDVAE_LIB; else export EBSDVAE_LIB=ebsd-vae_amd/lib/libebsdvae_$L.so; fi
  timeout -k 10 120 python3 tools/edge_micro.py --only net_end,net_end_valu 2>&1 | grep -v amdgpu.ids | sed "s/^/$L /" || exit 1
done; done
