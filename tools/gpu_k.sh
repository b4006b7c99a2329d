#!/bin/bash
# A/B (tests, micro, 3 bench pairs) then PMC passes over the weight-gradient micro cases.
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_ab.sh k fwd32,dgrad32,dgrad32u,dgrad32to64i,fwd32to64n,wgrad32 3 || exit 1
bash tools/pmc_conv.sh wg wgrad32,wgrad64,wgrad128 16 || exit 1
cat gpurun_out/pmc_wg_A.txt gpurun_out/pmc_wg_B.txt | cut -c1-600
