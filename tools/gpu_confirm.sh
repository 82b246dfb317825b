#!/bin/bash
# Full GPU suite + smoke + config B (driver command, no CPU leg): a quick confirmation of a default change.
set -u
O=gpurun_out/${OUT:-confirm}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu > $O/B.json 2> $O/B.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/B.err; exit $rc; }
python3 -c "import json;d=json.loads(open('$O/B.json').read().strip().splitlines()[-1]);s=d['single_pair'];print(round(d['value'],1), 'pairs/s; one pair', round(s['median_ms'],3), 'ms; knn', round(s['kernel_avg_ms']['k_knn_wave']*1e3,1), 'us; finish', round(s['kernel_avg_ms']['k_finish']*1e3,1), 'us; frac', round(d['roofline']['frac'],4))"
