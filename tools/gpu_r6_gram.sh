# round 6: first-conv statistics from the autocorrelation (13 displacements + border strips) -- parity, c4 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_first_fuse.py tests/test_gpu_fullsize.py tests/test_gpu_model.py > gpurun_out/r6_gram_tests.txt 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6_gram_tests.txt; exit 1; }
tail -1 gpurun_out/r6_gram_tests.txt; grep "moments:\|latents, moment" gpurun_out/r6_gram_tests.txt
for i in 1 2; do for L in default gram1; do
  if [ $L = default ]; then unset EBSDVAE_LIB; else export EBSDVAE_LIB=ebsd-vae_amd/lib/libebsdvae_$L.so; fi
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c5-steps 0 --steps 5 --warmup 2 --no-probe > gpurun_out/gram_$L.txt 2>/dev/null || exit 1
  echo "$L c4 $(python3 -c "import json;d=json.loads(open('gpurun_out/gram_$L.txt').read().splitlines()[-1]);c=d['c4_encoder_latents'];print(c['ms_per_batch'], c['engine_only']['value'])")"
done; done
