#!/bin/bash
set -u
O=gpurun_out/${OUT:-r06_fifo2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fifo_index.py tests/test_gpu_host_inputs.py tests/test_gpu_stream.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --no-cpu > $O/bench_B.out 2> $O/bench_B.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench_B.err; exit $rc; }
python3 -c "
import json;d=json.loads(open('$O/bench_B.out').read().strip().splitlines()[-1]);r=d['roofline'];h=d['host_handover']
print('B', round(d['value'],1), 'host', round(h['value'],1), 'index/reg', h['index_ms_per_registration'], 'single', d['single_pair']['median_ms'], 'kidx', d['single_pair']['kernel_avg_ms'].get('index'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_host -o run -- python3 bench.py --no-cpu --host-inputs --inflight 1 --no-fuse --steps 3 --warmup 1 --latency-pairs 3 --busy-steps 0 --no-verify > $O/kt_host.out 2> $O/kt_host.err
echo "kt rc=$?"
echo done
