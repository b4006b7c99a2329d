# Same-box A/B of variant libraries (python ebsd-vae_amd/build.py --variant NAME -D MACRO):
# VARIANTS="name ..." MTOOL=tools/conv_micro.py MARGS="--pieces 16 --only wgrad32" bash tools/gpu_ab_lib.sh
# two rounds of (micro case, 20-step bench) per library, default library first
cd $GRAFT_REPO_ROOT
for i in 1 2; do for L in default ${VARIANTS:-fnt}; do
  if [ $L = default ]; then unset EBSDVAE_LIB; else export EBSDVAE_LIB=ebsd-vae_amd/lib/libebsdvae_$L.so; fi
  timeout -k 10 120 python3 ${MTOOL:-tools/edge_micro.py} ${MARGS:---only first_valu} 2>&1 | grep -v amdgpu.ids | sed "s/^/$L /" || exit 1
  timeout -k 10 150 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 20 > gpurun_out/ab_$L.txt 2>/dev/null || exit 1
  echo "$L bench $(python3 -c "import json;d=json.loads(open('gpurun_out/ab_$L.txt').read().splitlines()[-1]);print(d['ms_per_step'])")"
done; done
