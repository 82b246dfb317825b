#!/bin/bash
# Round measurement set (outputs under gpurun_out/${OUT:-final}/): full GPU suite + smoke, the
# headline bench (driver command, CPU baselines), the stream / A / shipped-solver legs, a kernel
# trace of the driver command and of a one-pair-in-flight run (the roofline probe's regime), and
# the PMC traffic passes (FETCH_SIZE, WRITE_SIZE: separate runs, --kernel-trace only).
set -u
O=gpurun_out/${OUT:-final}
mkdir -p $O
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }
}
# PART=1: tests, smoke, the B (with its host hand-over leg), stream, stream-host and 2000-query B lines;
# PART=2: everything else (two gpurun calls); default both
P1=1; P2=1; [ "${PART:-0}" = 1 ] && P2=0; [ "${PART:-0}" = 2 ] && P1=0
if [ $P1 = 1 ]; then
[ "${SKIP_TESTS:-0}" = 1 ] || step gpu_tests 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
[ "${SKIP_TESTS:-0}" = 1 ] || step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench_B 600 python3 bench.py
step bench_stream 300 python3 bench.py --workload stream
step bench_stream_host 300 python3 bench.py --workload stream --no-cpu --host-inputs
step bench_B_q2000 400 python3 bench.py --queries 2000
fi
if [ $P2 = 1 ]; then
step bench_stream_ransac 500 python3 bench.py --workload stream --solver RANSAC_DRPM
step bench_A 400 python3 bench.py --workload A
step bench_A_ransac 400 python3 bench.py --workload A --solver RANSAC_DRPM
step bench_E 500 python3 bench.py --workload E
step kt_stream 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_stream -o run -- python3 bench.py --workload stream --no-cpu --steps 4 --warmup 1
step kt_driver 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_driver -o run -- python3 bench.py --no-cpu --no-host-leg
# the roofline fraction recomputed from the driver command's own kernel trace (tools/trace_frac.py)
f=$(find $O/kt_driver -name '*kernel_trace.csv' | head -1)
python3 tools/trace_frac.py $f $O/kt_driver.out > $O/kt_driver_frac.json && cat $O/kt_driver_frac.json
step kt_single 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_single -o run -- python3 bench.py --no-cpu --no-host-leg --inflight 1 --no-fuse --steps 5 --warmup 1
f=$(find $O/kt_single -name '*kernel_trace.csv' | head -1)
python3 tools/iter_profile.py $f > $O/per_iteration_single_pair.txt && cat $O/per_iteration_single_pair.txt
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c 300 rocprofv3 --kernel-trace --kernel-include-regex 'k_knn_wave|k_finish' --output-format csv \
      --pmc $c -d $O/pmc_$c -o run -- python3 bench.py --no-host-leg --steps 2 --warmup 1 --no-cpu --inflight 1 --no-fuse --latency-pairs 3
done
# the driver's N>1 launch shape at N=1 (torch.distributed.run, RCCL init, max-over-ranks timing)
step dist1 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu
fi
echo done
