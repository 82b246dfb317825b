#!/bin/bash
set -u
O=gpurun_out/${OUT:-groups}
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python3 bench.py "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc $(python3 -c "import json;d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]);print(round(d['value'],1))" 2>/dev/null)"; [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }
}
run B4g2 300 --no-cpu --latency-pairs 2 --inflight 4 --groups 2
run B6g3 300 --no-cpu --latency-pairs 2 --inflight 6 --groups 3
run B4g4 300 --no-cpu --latency-pairs 2 --inflight 4 --groups 4
run B6g6 300 --no-cpu --latency-pairs 2 --inflight 6 --groups 6
run B8g4 300 --no-cpu --latency-pairs 2 --inflight 8 --groups 4
run B3g3 300 --no-cpu --latency-pairs 2 --inflight 3 --groups 3
run S128g4 300 --workload stream --no-cpu --inflight 128 --groups 4
run S256g4 300 --workload stream --no-cpu --inflight 256 --groups 4
