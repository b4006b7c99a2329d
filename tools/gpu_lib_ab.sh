#!/bin/bash
# Same-box A/B of the in-tree library against a variant build (ebsd-vae_amd/lib/libebsdvae_VAR.so):
# optional parity tests (in-tree library), conv_micro cases for both, bench pairs alternating.
# Usage: bash tools/gpu_lib_ab.sh TAG VAR "pytest args|-" "micro cases|-" [pairs]
T=$1; V=$2; TESTS=$3; MICRO=$4; NP=${5:-2}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
NEW=ebsd-vae_amd/lib/libebsdvae.so; OLD=ebsd-vae_amd/lib/libebsdvae_$V.so
if [ "$TESTS" != "-" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -q -x --timeout 200 --timeout-method thread > $O/l_${T}_t.txt 2>&1; rc=$?
  tail -2 $O/l_${T}_t.txt; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/l_${T}_t.txt | head -20; exit $rc; }
fi
if [ "$MICRO" != "-" ]; then
  for L in new $V; do
    if [ $L = new ]; then LIB=$NEW; else LIB=$OLD; fi
    echo "== $L"
    EBSDVAE_LIB=$LIB timeout -k 10 200 python3 tools/conv_micro.py --pieces 16 --warm 0.5 --only $MICRO 2>&1 | grep -v amdgpu.ids; rc=${PIPESTATUS[0]}
    [ $rc -ne 0 ] && exit $rc
  done
fi
for i in $(seq 1 $NP); do
  for L in new $V; do
    if [ $L = new ]; then LIB=$NEW; else LIB=$OLD; fi
    EBSDVAE_LIB=$LIB timeout -k 10 150 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --c5-steps 0 --steps 20 > $O/l_${T}_${L}_$i.txt 2> $O/l_${T}_${L}_$i.err; rc=$?
    [ $rc -ne 0 ] && { tail -20 $O/l_${T}_${L}_$i.err; exit $rc; }
    echo "bench $L $i $(python3 -c "import json;d=json.loads(open('$O/l_${T}_${L}_$i.txt').read().splitlines()[-1]);print(d['ms_per_step'], d['value'], d['kernel_families_ms_per_step'])")"
  done
done
