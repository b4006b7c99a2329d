# round 6: idle gaps inside the plain training step at HEAD
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/trace_ab.sh r6g && python3 tools/step_gaps.py gpurun_out/tab_r6g 5 3 > gpurun_out/r6_gaps.txt 2>&1 && python3 tools/step_gaps.py gpurun_out/tab_r6g 6 3 >> gpurun_out/r6_gaps.txt 2>&1
rm -rf gpurun_out/tab_r6g
head -60 gpurun_out/r6_gaps.txt
