#!/bin/bash
# Sparse-leaf threshold sweep (IMLS_SPARSE: a leaf wanted by <= this many lanes is scanned per lane)
# on config B at the current defaults: pairs/s and the one-pair k_knn_wave average.
set -u
O=gpurun_out/${OUT:-sparse}
mkdir -p $O
export TMPDIR=/tmp
for sp in ${SPS:-32 16 24 48}; do
  IMLS_SPARSE=$sp timeout -k 10 300 python3 bench.py --no-cpu --steps 6 > $O/B_$sp.json 2> $O/B_$sp.err || exit $?
  python3 -c "import json;d=json.loads(open('$O/B_$sp.json').read().strip().splitlines()[-1]);s=d['single_pair'];print('sparse $sp', round(d['value'],1), 'pairs/s; one pair', round(s['median_ms'],3), 'ms; knn', round(s['kernel_avg_ms']['k_knn_wave']*1e3,1), 'us')"
done
