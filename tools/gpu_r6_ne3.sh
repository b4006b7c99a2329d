# round 6: net_end MFMA form, six-step unroll (no register rotation copies), branch-free g1 ring -- parity + micro
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py::test_network_end_matches_oracle \
  tests/test_gpu_trainer.py > gpurun_out/r6_ne3_tests.txt 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6_ne3_tests.txt; exit 1; }
tail -1 gpurun_out/r6_ne3_tests.txt
for i in 1 2; do timeout -k 10 120 python3 tools/edge_micro.py --only net_end,net_end_valu 2>&1 | grep -v amdgpu.ids || exit 1; done
