# round 6: first conv (training) with incremental pixel coordinates -- parity, micro and step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_trainer.py tests/test_gpu_first_fuse.py > gpurun_out/r6_fc_tests.txt 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6_fc_tests.txt; exit 1; }
tail -1 gpurun_out/r6_fc_tests.txt
for i in 1 2; do for L in default fc0; do
  if [ $L = default ]; then unset EBSDVAE_LIB; else export EBSDVAE_LIB=ebsd-vae_amd/lib/libebsdvae_$L.so; fi
  timeout -k 10 120 python3 tools/edge_micro.py --only first_valu 2>&1 | grep -v amdgpu.ids | sed "s/^/$L /" || exit 1
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 30 > gpurun_out/fc_$L.txt 2>/dev/null || exit 1
  echo "$L bench $(python3 -c "import json;d=json.loads(open('gpurun_out/fc_$L.txt').read().splitlines()[-1]);print(d['ms_per_step'])")"
done; done
