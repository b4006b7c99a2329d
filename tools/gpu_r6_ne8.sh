# round 6: net_end 64-row bands with 16-row running sums -- zero-bias residue on the saturated fixture
# (both band heights), parity, micro
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for L in default th32; do
  if [ $L = default ]; then unset EBSDVAE_LIB; else export EBSDVAE_LIB=ebsd-vae_amd/lib/libebsdvae_$L.so; fi
  timeout -k 10 200 python -u -m pytest -q -s --timeout 150 --timeout-method thread -m gpu "tests/test_gpu_trainer.py::test_trainer_forward_backward_vs_pinned_oracle" > gpurun_out/r6_ne8_res_$L.txt 2>&1
  echo "$L: $(tail -1 gpurun_out/r6_ne8_res_$L.txt)"; grep -E "^\[|decoder.13.0.bias" gpurun_out/r6_ne8_res_$L.txt | paste - - | sed "s/^/$L /"
done
unset EBSDVAE_LIB
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py::test_network_end_matches_oracle tests/test_gpu_trainer.py tests/test_gpu_fullsize.py tests/test_gpu_poison.py > gpurun_out/r6_ne8_tests.txt 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6_ne8_tests.txt; exit 1; }
tail -1 gpurun_out/r6_ne8_tests.txt
for i in 1 2; do for L in default th32; do
  if [ $L = default ]; then unset EBSDVAE_LIB; else export EBSDVAE_LIB=ebsd-vae_amd/lib/libebsdvae_$L.so; fi
  timeout -k 10 120 python3 tools/edge_micro.py --only net_end 2>&1 | grep -v amdgpu.ids | sed "s/^/$L /" || exit 1
done; done
