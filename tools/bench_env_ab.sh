#!/bin/bash
# Alternating bench.py runs across env settings (step time A/B):
#   bash tools/bench_env_ab.sh ROUNDS "VAR=a" "VAR=b" ...
export TMPDIR=/tmp
R=$1; shift
for i in $(seq "$R"); do
  for E in "$@"; do
    ms=$(env $E timeout -k 10 200 python3 bench.py --steps 30 --c4-batches 0 --c5-steps 0 --no-cpu-baseline 2>/dev/null \
         | python3 -c 'import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])["ms_per_step"])') || exit 1
    echo "$i $E $ms"
  done
done
