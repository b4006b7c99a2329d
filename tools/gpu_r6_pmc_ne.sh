# round 6: counters of the MFMA network end against the VALU form (tools/pmc_edge.sh)
R=$GRAFT_REPO_ROOT
cd $R
bash tools/pmc_edge.sh r6ne net_end,net_end_valu > gpurun_out/r6_pmc_ne.log 2>&1 || exit 1
cat gpurun_out/pmce_r6ne_A.txt gpurun_out/pmce_r6ne_B.txt > gpurun_out/r6_pmc_net_end.txt
rm -rf gpurun_out/pmce_r6ne_A gpurun_out/pmce_r6ne_B
