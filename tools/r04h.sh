set -u
O=gpurun_out/r04h; mkdir -p $O
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc $(python3 -c "import json;d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]);print(round(d['value'],1), d['unit'], (d.get('single_frame') or {}).get('median_ms'))" 2>/dev/null)"
  [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }
}
step stream 300 python3 bench.py --workload stream --no-cpu --latency-pairs 30
step stream_host 300 python3 bench.py --workload stream --no-cpu --host-inputs --latency-pairs 10
step B_host 300 python3 bench.py --no-cpu --host-inputs
step B_q2000 300 python3 bench.py --queries 2000 --no-cpu
step A 300 python3 bench.py --workload A --no-cpu
step dist1 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu
echo done
