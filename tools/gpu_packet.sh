#!/bin/bash
# Smaller traversal packets for the first ICP iterations (IMLS_PACKET / IMLS_PACKET_ITERS): parity of
# the projection tests at packet 32 and 16, then config B (driver command + the one-pair probe) per setting.
set -u
O=gpurun_out/${OUT:-packet}
mkdir -p $O
export TMPDIR=/tmp
for p in 32 16; do
  IMLS_PACKET=$p IMLS_PACKET_ITERS=20 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_verlet.py \
      tests/test_gpu_frames.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_$p.log 2>&1
  rc=$?; echo "tests packet $p rc=$rc"; tail -2 $O/tests_$p.log; [ $rc -eq 0 ] || exit $rc
done
for cfg in ${CFGS:-64:3 32:1 32:3 16:1 16:3}; do
  p=${cfg%%:*}; n=${cfg##*:}
  IMLS_PACKET=$p IMLS_PACKET_ITERS=$n timeout -k 10 300 python3 bench.py --no-cpu --steps 6 --warmup 2 > $O/B_${p}_$n.json 2> $O/B_${p}_$n.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 $O/B_${p}_$n.err; exit $rc; }
  python3 -c "import json;d=json.loads(open('$O/B_${p}_$n.json').read().strip().splitlines()[-1]);s=d['single_pair'];print('packet $p iters $n', round(d['value'],1), 'pairs/s; one pair', round(s['median_ms'],3), 'ms; knn', round(s['kernel_avg_ms']['k_knn_wave']*1e3,1), 'us; finish', round(s['kernel_avg_ms']['k_finish']*1e3,1), 'us')"
done
