#!/bin/bash
# Same-box knob A/B on the product library (outputs under gpurun_out/${OUT:-knobs}/):
#   TESTS="tests/a.py tests/b.py" TEST_ENV="IMLS_X=1"  — GPU tests first, with those knobs set;
#   KNOBS="base IMLS_X=1 IMLS_X=1+IMLS_Y=2"             — config B per knob set (base = none),
#   the whole list repeated ROUNDS times (alternating, so box drift hits every set alike).
# Each bench line: pairs/s, busy projection ms per step, one-pair k_knn_wave / k_finish, one pair.
set -u
O=gpurun_out/${OUT:-knobs}
mkdir -p $O
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-500} env ${TEST_ENV:-IMLS_NOTHING=0} python3 -u -m pytest $TESTS -m gpu -x -q --timeout 200 \
      --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
show() { python3 -c "
import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline'];sp=d.get('single_pair') or d.get('single_frame') or {};s=sp.get('kernel_avg_ms',{})
print('$2', round(d['value'],1), 'busy_proj', round(r.get('busy_projection_ms_per_step',0),2), 'knn', round(s.get('k_knn_wave',0)*1e3,1), 'finish', round(s.get('k_finish',0)*1e3,1), 'single', round(sp.get('median_ms',0),2), 'verify', d['verify']['mismatches'])"; }
for r in $(seq 1 ${ROUNDS:-2}); do
  kn=0
  for k in ${KNOBS:-base}; do
    f=$O/r${r}_$((++kn))
    envs=${k//+/ }; [ "$k" = base ] && envs="IMLS_NOTHING=0"
    timeout -k 10 300 env $envs python3 bench.py --no-cpu --steps ${STEPS:-8} --latency-pairs ${LAT:-10} ${BENCH_ARGS:-} > $f.json 2> $f.err \
      || { echo "bench $k failed"; tail -5 $f.err; exit 1; }
    show $f.json "$k r$r"
  done
done
echo done
