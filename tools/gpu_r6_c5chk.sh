# round 6: c5 re-check (two bench runs with the c5 leg only)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --strict-fp32-steps 0 --c4-batches 0 --steps 10 > gpurun_out/c5chk_$i.txt 2>gpurun_out/c5chk_$i.err || exit 1
  echo "run $i $(python3 -c "import json;d=json.loads(open('gpurun_out/c5chk_$i.txt').read().splitlines()[-1]);print(d['ms_per_step'], d['c5_256']['ms_per_step'])")"
done
