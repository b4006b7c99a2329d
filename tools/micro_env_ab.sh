#!/bin/bash
# A/B of conv_micro cases across env settings: bash tools/micro_env_ab.sh "CASES" "VAR=a" "VAR=b" ...
export TMPDIR=/tmp
C=$1; shift
for E in "$@"; do
  echo "== $E"
  env $E timeout -k 10 120 python3 tools/conv_micro.py --only $C || exit 1
done
