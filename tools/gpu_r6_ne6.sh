# round 6: net_end with 64-row bands -- parity (kernel, trainer, full size), then micro A/B against 32-row bands
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py::test_network_end_matches_oracle tests/test_gpu_trainer.py tests/test_gpu_fullsize.py > gpurun_out/r6_ne6_tests.txt 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6_ne6_tests.txt; exit 1; }
tail -1 gpurun_out/r6_ne6_tests.txt
for i in 1 2; do for L in default th32; do
  if [ $L = default ]; then unset EBSDVAE_LIB; else export EBSDVAE_LIB=ebsd-vae_amd/lib/libebsdvae_$L.so; fi
  timeout -k 10 120 python3 tools/edge_micro.py --only net_end,net_end_valu 2>&1 | grep -v amdgpu.ids | sed "s/^/$L /" || exit 1
done; done
