# round 6: level-1 slice reduction with 16-byte loads -- bitwise A/B of the step's gradient, tests, micro/step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 python3 tools/gflat_dump.py gpurun_out/g_new.npy && \
EBSDVAE_LIB=ebsd-vae_amd/lib/libebsdvae_red0.so timeout -k 10 120 python3 tools/gflat_dump.py gpurun_out/g_old.npy && \
python3 -c "import numpy as np; a=np.load('gpurun_out/g_new.npy'); b=np.load('gpurun_out/g_old.npy'); print('bitwise equal:', a.tobytes()==b.tobytes(), a.size)" || exit 1
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_trainer.py tests/test_gpu_determinism.py tests/test_gpu_kernels.py > gpurun_out/r6_red_tests.txt 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6_red_tests.txt; exit 1; }
tail -1 gpurun_out/r6_red_tests.txt
bash tools/gpu_trace.sh r6red adam_kernel 10 --steps 10 --c5-steps 0 --c4-batches 0 > /dev/null 2>&1; grep -i "reduce" gpurun_out/trace_r6red.txt | head -5; rm -rf gpurun_out/prof_r6red
for i in 1 2; do for L in default red0; do
  if [ $L = default ]; then unset EBSDVAE_LIB; else export EBSDVAE_LIB=ebsd-vae_amd/lib/libebsdvae_$L.so; fi
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 30 > gpurun_out/red_$L.txt 2>/dev/null || exit 1
  echo "$L bench $(python3 -c "import json;d=json.loads(open('gpurun_out/red_$L.txt').read().splitlines()[-1]);print(d['ms_per_step'])")"
done; done
