#!/bin/bash
# Per-layer serial profile of the in-tree library and of experiment builds
# (ebsd-vae_amd/lib/libebsdvae_<variant>.so, build.py --variant).
# Usage: bash tools/gpu_variants.sh TAG "variant1 variant2 ..." [grep-pattern]
T=${1:-var}; V=${2:-}; P=${3:-.}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out
cd $R
: > $O/var_$T.txt
for v in main $V; do
  if [ $v = main ]; then LIB=$R/ebsd-vae_amd/lib/libebsdvae.so; else LIB=$R/ebsd-vae_amd/lib/libebsdvae_$v.so; fi
  echo "== $v" >> $O/var_$T.txt
  EBSDVAE_LIB=$LIB timeout -k 10 200 python3 tools/layer_profile.py --serial > $O/var_${T}_$v.txt 2>&1 || { tail -20 $O/var_${T}_$v.txt; exit 1; }
  grep -E "$P" $O/var_${T}_$v.txt >> $O/var_$T.txt
done
cat $O/var_$T.txt
