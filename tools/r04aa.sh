set -u
O=gpurun_out/r04aa; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_inputs.py tests/test_gpu_stream.py tests/test_gpu_qfuse.py -x -q --timeout 200 --timeout-method thread > $O/tests.out 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.out; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for k in base IMLS_UPLOAD_CHUNKS=1 IMLS_UPLOAD_CHUNKS=8; do
    e=$k; [ $k = base ] && e=IMLS_NOTHING=0
    timeout -k 10 300 env $e python3 bench.py --workload stream --no-cpu --host-inputs --steps 6 --latency-pairs 40 > $O/s_${r}_${k//=/_}.json 2> $O/s_${r}_${k//=/_}.err || { echo "bench $k failed"; tail -3 $O/s_${r}_${k//=/_}.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('$O/s_${r}_${k//=/_}.json').read().strip().splitlines()[-1]);sf=d['single_frame'];print('r$r $k', round(d['value'],1), 'single', round(sf['median_ms'],3), round(sf['p90_ms'],3), 'hand-over', round(sf['host_handover_median_ms'],3), 'verify', d['verify']['mismatches'])"
  done
done
