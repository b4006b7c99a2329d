# round 6: moment-based first-conv statistics for the inference path -- parity, then c4 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_first_fuse.py tests/test_gpu_model.py -k "first or encoder_only" -s > gpurun_out/r6_c4_tests.txt 2>&1 || { echo TESTS_FAILED; exit 1; }
for v in on off gram0 on2; do
  case $v in off) E="EBSDVAE_FIRST_FUSE=0";; gram0) E="EBSDVAE_FIRST_GRAM=0";; *) E="";; esac
  env $E timeout -k 10 200 python bench.py --no-cpu-baseline --strict-fp32-steps 0 --c5-steps 0 --steps 4 --warmup 2 --no-probe > gpurun_out/r6_c4_$v.json 2> gpurun_out/r6_c4_$v.err || exit 1
done
bash tools/gpu_trace.sh r6c4b heads_fwd 20 --steps 2 --warmup 1 --c5-steps 0 --c4-batches 30 > /dev/null
rm -rf gpurun_out/prof_r6c4b
