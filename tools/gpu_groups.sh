#!/bin/bash
# Launch-group sweep (outputs under gpurun_out/${OUT:-r03_groups}/): each RUNS entry is
# NAME:bench-args ('_' for spaces), e.g. "s2048g2:--workload_stream_--inflight_2048_--groups_2".
O=gpurun_out/${OUT:-r03_groups}; mkdir -p $O; export TMPDIR=/tmp
run() { n=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }; python3 -c "
import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);r=d['roofline']
print('$n', round(d['value'],1), 'ms/step', round(d['ms_per_step'],2), 'busy_proj', round(r.get('busy_projection_ms_per_step',0),2), 'any', round(r.get('busy_any_ms_per_step',0),2))"; grep "host time" $O/$n.err || true; }
for e in ${RUNS:-}; do run ${e%%:*} $(echo ${e#*:} | tr '_' ' '); done
echo done
