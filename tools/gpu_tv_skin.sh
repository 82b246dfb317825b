#!/bin/bash
# TV skin lists: parity (tests/test_gpu_tv.py), then config E at several skins (IMLS_TV_SKIN).
set -u
O=gpurun_out/${OUT:-tvskin}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_tv.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for sk in ${SKINS:-0 0.015 0.03 0.06}; do
  IMLS_TV_SKIN=$sk timeout -k 10 300 python3 bench.py --workload E --no-cpu > $O/E_$sk.json 2> $O/E_$sk.err
  rc=$?; echo "skin $sk rc=$rc $(python3 -c "import json;d=json.loads(open('$O/E_$sk.json').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['achieved'])")"; [ $rc -eq 0 ] || exit $rc
done
