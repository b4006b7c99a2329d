#!/bin/bash
# f16x3 parity subset, then an A/B of the conv arithmetic (bench without c4 / c5 / CPU legs)
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -k "f16" > gpurun_out/t_f16.txt 2>&1 || { tail -40 gpurun_out/t_f16.txt; exit 1; }
tail -2 gpurun_out/t_f16.txt
for p in ${PRECS:-f16x3 bf16x6 f16x3 bf16x6}; do
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --c4-batches 0 --c5-steps 0 --precision $p > gpurun_out/b_$p.txt 2>&1 || { tail -20 gpurun_out/b_$p.txt; exit 1; }
python3 -c "import json,sys;d=json.loads(open('gpurun_out/b_$p.txt').read().strip().splitlines()[-1]);print('$p',d['value'],d['ms_per_step'],d['roofline']['frac'],d['kernel_families_ms_per_step'])"
done
