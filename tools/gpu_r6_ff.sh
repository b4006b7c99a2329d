set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_first_fuse.py -s > gpurun_out/r6_ff_tests.txt 2>&1 || { echo TESTS_FAILED; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --strict-fp32-steps 0 > gpurun_out/r6_ff_on.json 2> gpurun_out/r6_ff_on.err && \
EBSDVAE_FIRST_FUSE=0 timeout -k 10 300 python bench.py --no-cpu-baseline --strict-fp32-steps 0 > gpurun_out/r6_ff_off.json 2> gpurun_out/r6_ff_off.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --strict-fp32-steps 0 > gpurun_out/r6_ff_on2.json 2> gpurun_out/r6_ff_on2.err
