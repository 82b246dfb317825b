#!/bin/bash
set -u
O=gpurun_out/rs; mkdir -p $O; export TMPDIR=/tmp
for r in 0.25 2 16 1000000; do
  IMLS_RESEED=$r timeout -k 10 300 python3 bench.py --no-cpu --latency-pairs 2 > $O/B_$r.json 2> $O/B_$r.err
  rc=$?; echo "reseed $r rc=$rc $(python3 -c "import json;d=json.loads(open('$O/B_$r.json').read().strip().splitlines()[-1]);print(d['value'], d['single_pair']['median_ms'])")"; [ $rc -eq 0 ] || exit $rc
done
