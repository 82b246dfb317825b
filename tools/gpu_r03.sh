#!/bin/bash
# Round-3 combined GPU call (outputs under gpurun_out/${OUT:-r03}/): the GPU test suite (all tests,
# no -x: the perf steps run even if a test fails), smoke, the headline bench (with the CPU legs),
# a same-box A/B of the product library against csrc/variant/libimls_gpu.so, knob variants of the
# product library (KNOBS), and the debug build's per-wave traversal records.
set -u
O=gpurun_out/${OUT:-r03}
mkdir -p $O
export TMPDIR=/tmp
fail=0
step() {  # name, timeout, command... (a time limit / abort / fault ends the script)
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"
  if [ $rc -ge 124 ]; then tail -5 $O/$name.err; exit $rc; fi
  [ $rc -eq 0 ] || { fail=1; tail -8 $O/$name.out; tail -5 $O/$name.err; }
}
show() { python3 -c "
import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline'];s=(r.get('serialised_single_pair') or {}).get('kernel_avg_ms',{})
print('$2', round(d['value'],1), 'frac', round(r['frac'],4), 'busy_proj', round(r.get('busy_projection_ms_per_step',0),2), 'knn', round(s.get('k_knn_wave',0)*1e3,1), 'finish', round(s.get('k_finish',0)*1e3,1), 'single', round((d.get('single_pair') or {}).get('median_ms',0),2))" || true; }
[ "${SKIP_TESTS:-0}" = 1 ] || step gpu_tests 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
[ "${SKIP_TESTS:-0}" = 1 ] || step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
[ "${SKIP_BENCH:-0}" = 1 ] || { step bench 400 python3 bench.py; show $O/bench.out bench; }
for w in ${EXTRA:-}; do   # extra bench legs: WORKLOAD or WORKLOAD+SOLVER (e.g. stream A A+RANSAC_DRPM E)
  wl=${w%%+*}; sv=LS; [ "$w" != "$wl" ] && sv=${w#*+}
  step bench_$w 400 python3 bench.py --workload $wl --solver $sv; show $O/bench_$w.out "bench $w"
done
V=planetary-lidar-odometry_amd/csrc/variant/libimls_gpu.so
for r in $(seq 1 ${ROUNDS:-1}); do
  [ -f $V ] || break
  step base_$r 200 python3 bench.py --no-cpu --steps 8 --latency-pairs 10; show $O/base_$r.out "base $r"
  step var_$r 200 env IMLS_LIB_PATH=$V python3 bench.py --no-cpu --steps 8 --latency-pairs 10; show $O/var_$r.out "variant $r"
done
for k in ${KNOBS:-}; do   # NAME=VALUE, several joined by '+'
  step knob_$k 200 env ${k//+/ } python3 bench.py --no-cpu --steps 8 --latency-pairs 10; show $O/knob_$k.out "$k"
done
[ "${SKIP_DUMP:-0}" = 1 ] || step wave_dump 240 env IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/debug/libimls_gpu.so python3 tools/wave_dump.py 1 2 3 6
echo "done fail=$fail"
