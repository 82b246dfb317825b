#!/bin/bash
# Round 6: more launch sequences in flight with more hardware queues (IMLS_BENCH_HW_QUEUES) — same box
set -u
O=gpurun_out/${OUT:-r06_hwq}
mkdir -p $O
export TMPDIR=/tmp
show() { python3 -c "
import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline']
print('$2', round(d['value'],1), 'ms/step', round(d['ms_per_step'],3), 'busy_proj', round(r.get('busy_projection_ms_per_step',0),2))"; }
for r in 1 2; do
  for cfg in "8 4 4" "16 4 4" "16 5 5" "16 6 6" "16 8 8" "32 8 8"; do
    set -- $cfg
    f=$O/B_q$1_p$2_g$3_$r
    IMLS_BENCH_HW_QUEUES=$1 timeout -k 10 300 python3 bench.py --no-cpu --no-host-leg --steps 8 --latency-pairs 3 --inflight $2 --groups $3 > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    show $f.json "hwq $1 inflight $2 groups $3 round $r"
  done
done
echo done
