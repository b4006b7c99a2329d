# round 6: where the 8x8 / 16x16 convs' time goes: batch scaling, one- vs two-image tiles, timing-only builds
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
C=fwd128s8,dgrad128s8,fwd128s16
for Bt in 256 1024; do
  timeout -k 10 150 python3 tools/conv_micro.py --pieces 16 --warm 0.5 --batch $Bt --only $C 2>&1 | grep -v amdgpu.ids | sed "s/^/B$Bt /" || exit 1
done
EBSDVAE_CONV_SMALL1=0 timeout -k 10 150 python3 tools/conv_micro.py --pieces 16 --warm 0.5 --only $C 2>&1 | grep -v amdgpu.ids | sed "s/^/two-image /" || exit 1
for L in nomfma2 nostage; do
  EBSDVAE_LIB=ebsd-vae_amd/lib/libebsdvae_$L.so timeout -k 10 150 python3 tools/conv_micro.py --pieces 16 --warm 0.5 --only $C 2>&1 | grep -v amdgpu.ids | sed "s/^/$L /" || exit 1
done
