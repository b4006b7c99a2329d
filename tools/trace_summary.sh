#!/bin/bash
# per-family ms/step from a traced 13-step bench (tools/gpu_quick.sh)
python tools/pmc_traffic.py --trace gpurun_out/tr_$1 --steps 13 --out /tmp/s_$1.json > /dev/null && python -c "
import json; d=json.load(open('/tmp/s_$1.json'))['trace']
for k,v in sorted(d.items(), key=lambda kv:-kv[1]['ms_per_step']): print(f'{k:16s} {v[\"ms_per_step\"]:7.3f} ms  {v[\"launches\"]//13:4d} launches  {v[\"avg_launch_us\"]:8.2f} us')"
