#!/bin/bash
# Round 6 closing check on the final tree: the GPU suite, smoke, and the driver's plain bench command.
set -u
O=gpurun_out/${OUT:-r06_check}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.out 2> $O/gpu_tests.err
rc=$?; echo "tests rc=$rc"; tail -2 $O/gpu_tests.out; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.out 2> $O/smoke.err; echo "smoke rc=$?"; cat $O/smoke.out
timeout -k 10 600 python3 bench.py > $O/bench.out 2> $O/bench.err; echo "bench rc=$?"
python3 -c "
import json;d=json.loads(open('$O/bench.out').read().strip().splitlines()[-1]);r=d['roofline'];h=d['host_handover'];c=d['cpu_baseline']
print(round(d['value'],1), 'host', round(h['value'],1), 'frac', round(r['frac'],4), 'traffic', r['traffic'], r['traffic_meta'].get('calibrated'), 'cpu', c['value'])"
echo done
