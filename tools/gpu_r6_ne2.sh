# round 6: one-barrier MFMA network end -- parity, micro timing, counters
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "network_end" -s > gpurun_out/r6_ne2_tests.txt 2>&1 || { echo TESTS_FAILED; exit 1; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_trainer.py -k "vae128_b8_c1 or vae256 or fusion" -s >> gpurun_out/r6_ne2_tests.txt 2>&1 || { echo TESTS2_FAILED; exit 1; }
timeout -k 10 120 python tools/edge_micro.py --only net_end,net_end_valu > gpurun_out/r6_ne2_micro.txt 2>&1 && \
EBSDVAE_LIB=$R/ebsd-vae_amd/lib/libebsdvae_firstpk.so timeout -k 10 200 python tools/conv_micro.py --pieces 16 --only fwd32poolx --batch 1024 > gpurun_out/r6_micro_first2.txt 2>&1 && \
timeout -k 10 200 python tools/conv_micro.py --pieces 16 --only fwd32pool,fwd32poolx --batch 1024 >> gpurun_out/r6_micro_first2.txt 2>&1 && \
bash tools/pmc_edge.sh r6ne2 net_end > gpurun_out/r6_pmc_ne2.log 2>&1 && \
cat gpurun_out/pmce_r6ne2_A.txt gpurun_out/pmce_r6ne2_B.txt > gpurun_out/r6_pmc_net_end2.txt
rm -rf gpurun_out/pmce_r6ne2_A gpurun_out/pmce_r6ne2_B
