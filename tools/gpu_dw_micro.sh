# fused input+weight gradient (conv_fused.hip) vs the separate kernels, and variant libraries
# built with `python ebsd-vae_amd/build.py --variant NAME -D MACRO` (names as arguments)
cd $GRAFT_REPO_ROOT
echo "== base"; timeout -k 10 200 python3 tools/conv_micro.py --pieces 16 --warm 0.5 --only dwgrad32,dwgrad32u,dgrad32,wgrad32,dgrad32u,wgrad32u 2>&1 | grep -v amdgpu.ids || exit 1
for v in "$@"; do echo "== $v"; EBSDVAE_LIB=ebsd-vae_amd/lib/libebsdvae_$v.so timeout -k 10 120 python3 tools/conv_micro.py --pieces 16 --warm 0.5 --only dwgrad32,dwgrad32u 2>&1 | grep -v amdgpu.ids || exit 1; done
