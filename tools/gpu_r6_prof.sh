# round 6: where the fused first conv's time goes -- micro A/B and serial traces of c4 / c2
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 200 python tools/conv_micro.py --pieces 16 --only fwd32pool,fwd32poolx,fwd32 > $O/r6_micro_first.txt 2>&1 && \
timeout -k 10 200 python tools/conv_micro.py --pieces 16 --batch 1024 --only fwd32pool,fwd32poolx >> $O/r6_micro_first.txt 2>&1 && \
bash tools/gpu_trace.sh r6c4 heads_fwd 20 --steps 2 --warmup 1 --c5-steps 0 --c4-batches 30 > /dev/null && \
bash tools/gpu_trace.sh r6c2 adam_kernel 10 --steps 20 --c5-steps 0 --c4-batches 0 > /dev/null
rm -rf $O/prof_r6c4 $O/prof_r6c2
