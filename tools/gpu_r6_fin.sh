# round 6: the encoder's last reduction batch on the main stream after one join -- tests, step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_trainer.py tests/test_gpu_determinism.py tests/test_gpu_dp.py tests/test_gpu_model.py tests/test_gpu_poison.py > gpurun_out/r6_fin_tests.txt 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6_fin_tests.txt; exit 1; }
tail -1 gpurun_out/r6_fin_tests.txt
for i in 1 2 3; do for S in 0 1; do
  EBSDVAE_FINAL_REDUCE_SIDE=$S timeout -k 10 200 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 40 > gpurun_out/fin_$S.txt 2>/dev/null || exit 1
  echo "final_on_side=$S bench $(python3 -c "import json;d=json.loads(open('gpurun_out/fin_$S.txt').read().splitlines()[-1]);print(d['ms_per_step'])")"
done; done
