# round 6: net_end running sums folded every 8 rows instead of 16 -- residue on the saturated fixture, micro
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for L in default fold8; do
  if [ $L = default ]; then unset EBSDVAE_LIB; else export EBSDVAE_LIB=ebsd-vae_amd/lib/libebsdvae_$L.so; fi
  timeout -k 10 200 python -u -m pytest -q -s --timeout 150 --timeout-method thread -m gpu "tests/test_gpu_trainer.py::test_trainer_forward_backward_vs_pinned_oracle" -k edge > gpurun_out/r6_fold_$L.txt 2>&1
  echo "$L: $(tail -1 gpurun_out/r6_fold_$L.txt)"; grep -E "decoder.13.0.bias" gpurun_out/r6_fold_$L.txt | sed "s/^/$L /"
done
for i in 1 2; do for L in default fold8; do
  if [ $L = default ]; then unset EBSDVAE_LIB; else export EBSDVAE_LIB=ebsd-vae_amd/lib/libebsdvae_$L.so; fi
  timeout -k 10 120 python3 tools/edge_micro.py --only net_end 2>&1 | grep -v amdgpu.ids | sed "s/^/$L /" || exit 1
done; done
