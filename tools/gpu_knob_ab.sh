#!/bin/bash
# Same-box A/B of env knobs on the product library (outputs under gpurun_out/${OUT:-kab}/): optional
# GPU tests first (TESTS="tests/test_x.py ..."), then config B (BENCH_ARGS) alternated ROUNDS times
# between the defaults ("base") and every KNOBS entry (NAME=VALUE, several joined by '+').
set -u
O=gpurun_out/${OUT:-kab}
mkdir -p $O
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-500} python3 -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
show() { python3 -c "
import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline'];s=(r.get('serialised_single_pair') or {}).get('kernel_avg_ms',{})
print('$2', round(d['value'],1), 'busy_proj', round(r.get('busy_projection_ms_per_step',0),2), 'knn', round(s.get('k_knn_wave',0)*1e3,1), 'finish', round(s.get('k_finish',0)*1e3,1), 'single', round((d.get('single_pair') or {}).get('median_ms',0),2), 'verify', d['verify']['mismatches'])"; }
for r in $(seq 1 ${ROUNDS:-2}); do
  for k in base ${KNOBS:-}; do
    envs=""; [ "$k" = base ] || envs="${k//+/ }"
    timeout -k 10 300 env $envs python3 bench.py --no-cpu --steps ${STEPS:-8} --latency-pairs 10 ${BENCH_ARGS:-} > $O/${k}_$r.json 2> $O/${k}_$r.err
    rc=$?; [ $rc -eq 0 ] || { echo "$k rc=$rc"; tail -5 $O/${k}_$r.err; exit $rc; }
    show $O/${k}_$r.json "$k $r"
  done
done
echo done
