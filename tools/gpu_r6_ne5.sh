# round 6: net_end at HEAD vs the working tree, same box
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py::test_network_end_matches_oracle tests/test_gpu_trainer.py > gpurun_out/r6_ne5_tests.txt 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6_ne5_tests.txt; exit 1; }
tail -1 gpurun_out/r6_ne5_tests.txt
for i in 1 2; do for L in default head neu2 nebr; do
  if [ $L = default ]; then unset EBSDVAE_LIB; else export EBSDVAE_LIB=ebsd-vae_amd/lib/libebsdvae_$L.so; fi
  timeout -k 10 120 python3 tools/edge_micro.py --only net_end 2>&1 | grep -v amdgpu.ids | sed "s/^/$L /" || exit 1
done; done
