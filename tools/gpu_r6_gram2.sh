# round 6: first-conv statistics kernels alone (B = 256 and 1024), new vs previous form
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2; do for L in default gram1; do
  if [ $L = default ]; then unset EBSDVAE_LIB; else export EBSDVAE_LIB=ebsd-vae_amd/lib/libebsdvae_$L.so; fi
  for Bt in 256 1024; do
    timeout -k 10 120 python3 tools/edge_micro.py --batch $Bt --only first_stats,first_valu 2>&1 | grep -v amdgpu.ids | sed "s/^/$L B$Bt /" || exit 1
  done
done; done
