# round 6: counters of the final net_end (64-row bands, six-step unroll) -- tools/pmc_edge.sh
R=$GRAFT_REPO_ROOT
cd $R
bash tools/pmc_edge.sh r6ne3 net_end > gpurun_out/r6_pmc_ne3.log 2>&1 || exit 1
cat gpurun_out/pmce_r6ne3_A.txt gpurun_out/pmce_r6ne3_B.txt > gpurun_out/r6_pmc_net_end3.txt
rm -rf gpurun_out/pmce_r6ne3_A gpurun_out/pmce_r6ne3_B
cat gpurun_out/r6_pmc_net_end3.txt
