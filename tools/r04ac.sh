set -u
O=gpurun_out/r04ac; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --workload stream --no-cpu --host-inputs > $O/bench_stream_host.out 2> $O/bench_stream_host.err
rc=$?; echo "stream host rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json;d=json.loads(open('$O/bench_stream_host.out').read().strip().splitlines()[-1]);sf=d['single_frame'];print('stream host', round(d['value'],1), 'single', round(sf['median_ms'],3), round(sf['p90_ms'],3), 'hand-over', round(sf['host_handover_median_ms'],3), 'verify', d['verify']['mismatches'])"
