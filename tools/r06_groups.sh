#!/bin/bash
# Round 6: config B launch-shape knobs on the current kernels (same box): pairs in flight x launch
# sequences (groups), 2 rounds each.
set -u
O=gpurun_out/${OUT:-r06_groups}
mkdir -p $O
export TMPDIR=/tmp
show() { python3 -c "
import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline']
print('$2', round(d['value'],1), 'ms/step', round(d['ms_per_step'],3), 'busy_proj', round(r.get('busy_projection_ms_per_step',0),2))"; }
for r in 1 2; do
  for cfg in "4 4" "4 2" "8 4" "6 6" "3 3"; do
    set -- $cfg
    f=$O/B_p$1_g$2_$r
    timeout -k 10 300 python3 bench.py --no-cpu --no-host-leg --steps 8 --latency-pairs 3 --inflight $1 --groups $2 > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    show $f.json "inflight $1 groups $2 round $r"
  done
done
echo done
