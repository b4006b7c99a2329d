# round 6: fused first conv + MFMA network end -- parity, micro timing, bench A/B (one box)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_first_fuse.py tests/test_gpu_kernels.py -k "first_fuse or network_end" -s \
  > gpurun_out/r6_ff_tests.txt 2>&1 || { echo TESTS_FAILED; exit 1; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_trainer.py tests/test_gpu_determinism.py tests/test_gpu_fullsize.py -s \
  > gpurun_out/r6_ff_tests2.txt 2>&1 || { echo TESTS2_FAILED; exit 1; }
timeout -k 10 120 python tools/edge_micro.py --only net_end,net_end_valu > gpurun_out/r6_ne_micro.txt 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --strict-fp32-steps 0 > gpurun_out/r6_ff_on.json 2> gpurun_out/r6_ff_on.err && \
EBSDVAE_FIRST_FUSE=0 EBSDVAE_NET_END_MFMA=0 timeout -k 10 300 python bench.py --no-cpu-baseline --strict-fp32-steps 0 > gpurun_out/r6_ff_off.json 2> gpurun_out/r6_ff_off.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --strict-fp32-steps 0 > gpurun_out/r6_ff_on2.json 2> gpurun_out/r6_ff_on2.err
