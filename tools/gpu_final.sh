#!/bin/bash
# Round-3 closing run: the whole GPU suite at HEAD, then the profile set (tools/prof_r03.sh).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_final.txt 2>&1 || { tail -40 $O/t_final.txt; exit 1; }
tail -1 $O/t_final.txt
bash tools/prof_r03.sh || exit 1
EBSDVAE_LIB=$R/ebsd-vae_amd/lib/libebsdvae_cvtrace.so timeout -k 10 200 python3 tools/conv_micro.py --pieces 16 --warm 0.3 --only fwd32,dgrad32,dgrad32u,fwd64,dgrad64,fwd128,dgrad128 > $O/trace_final.txt 2>&1 || exit 1
echo all done
