#!/bin/bash
# conv_micro over the experiment builds: bash tools/micro_variants.sh TAG "cases" "variant1 variant2 ..." [pieces]
T=$1; C=$2; V=$3; P=${4:-16}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
: > $R/gpurun_out/mv_$T.txt
for v in base $V; do
  if [ $v = base ]; then L=$R/ebsd-vae_amd/lib/libebsdvae.so; else L=$R/ebsd-vae_amd/lib/libebsdvae_$v.so; fi
  echo "== $v" >> $R/gpurun_out/mv_$T.txt
  EBSDVAE_LIB=$L timeout -k 10 200 python3 $R/tools/conv_micro.py --pieces $P --warm 0.5 --only $C >> $R/gpurun_out/mv_$T.txt 2>&1 || exit 1
done
echo ok
