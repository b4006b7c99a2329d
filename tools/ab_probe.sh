export TMPDIR=/tmp
for i in 1 2 3 4; do
  for F in "" "--no-probe"; do
    ms=$(timeout -k 10 200 python3 bench.py --steps 30 --c4-batches 0 --c5-steps 0 --no-cpu-baseline $F 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])["ms_per_step"])') || exit 1
    echo "$i probe$F $ms"
  done
done
