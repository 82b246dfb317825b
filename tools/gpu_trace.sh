#!/bin/bash
# Kernel traces of the driver command (config B) and of the stream leg (outputs under
# gpurun_out/${OUT:-trace}/): rocprofv3 --kernel-trace --stats; tools/trace_busy.py over the timed
# window prints the union busy time and the largest idle gaps.
set -u
O=gpurun_out/${OUT:-trace}
mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_B:-0}" != 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/B -o run -- python3 bench.py --no-cpu > $O/B.json 2> $O/B.err
  rc=$?; echo "trace B rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/B.err; exit $rc; }
  f=$(find $O/B -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_frac.py $f $O/B.json > $O/B_frac.json; cat $O/B_frac.json
  python3 tools/trace_busy.py $f 0 0 > $O/B_busy.txt
fi
if [ "${SKIP_STREAM:-0}" != 1 ]; then
  IMLS_DEBUG_HOST=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stream -o run -- python3 bench.py --workload stream --no-cpu --steps 4 --busy-steps 0 > $O/stream.json 2> $O/stream.err
  rc=$?; echo "trace stream rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/stream.err; exit $rc; }
  f=$(find $O/stream -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_busy.py $f 0.6 25 > $O/stream_busy.txt; head -50 $O/stream_busy.txt
  python3 tools/trace_frac.py $f $O/stream.json --busy-steps 0 > $O/stream_frac.json; cat $O/stream_frac.json
fi
echo done
