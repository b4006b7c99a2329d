#!/bin/bash
# Whole GPU suite at HEAD, then the A/B against libebsdvae_old.so (micro + 3 bench pairs).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_full_n.txt 2>&1 || { tail -30 $O/t_full_n.txt; exit 1; }
tail -1 $O/t_full_n.txt
bash tools/gpu_ab.sh n fwd32,dgrad32,dgrad32u,dgrad64,dgrad128,dgrad32to64i 3
EBSDVAE_LIB=$R/ebsd-vae_amd/lib/libebsdvae_cvtrace.so timeout -k 10 200 python3 tools/conv_micro.py --pieces 16 --warm 0.3 --only fwd32,dgrad32,dgrad32u,fwd64,dgrad64,fwd128,dgrad128 > $O/trace_n.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/trace_n.txt
