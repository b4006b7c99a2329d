#!/bin/bash
# A/B of conv_micro cases across experiment builds: bash tools/micro_ab.sh "CASES" lib1 lib2 ...
export TMPDIR=/tmp
C=$1; shift
for L in "$@"; do
  echo "== $L"
  EBSDVAE_LIB=$GRAFT_REPO_ROOT/ebsd-vae_amd/lib/$L timeout -k 10 120 python3 tools/conv_micro.py --only $C || exit 1
done
