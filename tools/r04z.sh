set -u
O=gpurun_out/r04z; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_qfuse.py tests/test_gpu_stream.py tests/test_gpu_frames.py tests/test_gpu_parity.py tests/test_gpu_verlet.py -x -q --timeout 200 --timeout-method thread > $O/tests.out 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.out; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for k in base IMLS_SOURCE_RADIX=1; do
    e=$k; [ $k = base ] && e=IMLS_NOTHING=0
    timeout -k 10 100 env $e python3 tools/frame_probe.py 30 > $O/probe_${r}_${k//=/_}.txt 2>&1 || { echo "probe failed"; exit 1; }
    echo "r$r $k: $(head -1 $O/probe_${r}_${k//=/_}.txt)"
  done
done
timeout -k 10 300 python3 bench.py --workload stream --no-cpu > $O/bench_stream.out 2> $O/bench_stream.err
rc=$?; echo "stream rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json;d=json.loads(open('$O/bench_stream.out').read().strip().splitlines()[-1]);sf=d['single_frame'];print('stream', round(d['value'],1), 'single', round(sf['median_ms'],3), round(sf['p90_ms'],3), 'hand-over', round(sf['host_handover_median_ms'],3), 'verify', d['verify']['mismatches'])"
