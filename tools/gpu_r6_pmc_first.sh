# round 6: counters of the first block's backward pass (in_bwd_edge_kernel<FUSE_FIRST_RC>) and the apply
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 python3 tools/edge_micro.py --only first_rc,in_apply,ref_copy 2>&1 | grep -v amdgpu.ids
bash tools/pmc_edge.sh r6fr first_rc,in_apply > gpurun_out/r6_pmc_fr.log 2>&1 || exit 1
cat gpurun_out/pmce_r6fr_A.txt gpurun_out/pmce_r6fr_B.txt | grep -v "at::native" > gpurun_out/r6_pmc_first.txt
rm -rf gpurun_out/pmce_r6fr_A gpurun_out/pmce_r6fr_B
cat gpurun_out/r6_pmc_first.txt
