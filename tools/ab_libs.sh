#!/bin/bash
# Same-box A/B of several libraries (outputs under gpurun_out/${OUT:-ab}/): config B (BENCH_ARGS) for
# the product library and each csrc/var_NAME/libimls_gpu.so named in VARS, alternated ROUNDS times;
# one line per run: pairs/s, busy projection ms per step, one-pair k_knn_wave / k_finish µs.
set -u
O=gpurun_out/${OUT:-ab}
mkdir -p $O
export TMPDIR=/tmp
C=planetary-lidar-odometry_amd/csrc
show() { python3 -c "
import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline'];s=r.get('serialised_single_pair',{}).get('kernel_avg_ms',{})
sp=d.get('single_pair') or {}
print('$2', round(d['value'],1), 'busy_proj', round(r.get('busy_projection_ms_per_step',0),2), 'knn', round(s.get('k_knn_wave',0)*1e3,1), 'finish', round(s.get('k_finish',0)*1e3,1), 'single', round(sp.get('median_ms',0),2))"; }
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in product ${VARS:-}; do
    lib=""; [ $v = product ] || lib=$C/var_$v/libimls_gpu.so
    f=$O/${v}_$r
    env ${lib:+IMLS_LIB_PATH=$lib} timeout -k 10 300 python3 bench.py --no-cpu --steps ${STEPS:-8} --latency-pairs 10 ${BENCH_ARGS:-} > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    show $f.json "$v $r"
  done
done
echo done
