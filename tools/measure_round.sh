#!/bin/bash
# Round measurement set (outputs under gpurun_out/${OUT:-final}/).
# PART=1: the FETCH_SIZE calibration kernels (tools/calib) and the PMC FETCH / WRITE passes of the
#         projection kernels FIRST (separate --pmc runs, --kernel-trace only), the traffic figure from
#         them (tools/pmc_traffic.py → $O/pmc_traffic.json), then the GPU suite, smoke, and the B line
#         reading THIS run's traffic file, its 2000-query variant, the stream legs;
# PART=2: the other legs (shipped solver stream with its CPU baseline, A, A-RANSAC, E), the kernel traces
#         of the driver command and of one pair in flight, the torchrun N=1 launch.  Default: both.
set -u
O=gpurun_out/${OUT:-final}
mkdir -p $O $O/cal
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }
}
P1=1; P2=1; [ "${PART:-0}" = 1 ] && P2=0; [ "${PART:-0}" = 2 ] && P1=0
if [ $P1 = 1 ]; then
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/cal/fetch -o run -- tools/calib/gather_cal > $O/cal/fetch.out 2> $O/cal/fetch.err; echo "cal fetch rc=$?"
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/cal/write -o run -- tools/calib/gather_cal > $O/cal/write.out 2> $O/cal/write.err; echo "cal write rc=$?"
python3 tools/calib/gather_cal.py $O/cal > $O/cal/cal.txt 2>&1; echo "cal rc=$?"
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c 300 rocprofv3 --kernel-trace --kernel-include-regex 'k_knn_wave|k_finish' --output-format csv \
      --pmc $c -d $O/pmc_$c -o run -- python3 bench.py --no-host-leg --steps 2 --warmup 1 --no-cpu --inflight 1 --no-fuse --latency-pairs 3
done
python3 tools/pmc_traffic.py $O $O/profile_copy $O/cal/gather_cal.json > $O/pmc_traffic.txt 2>&1; echo "traffic rc=$?"
[ "${SKIP_TESTS:-0}" = 1 ] || step gpu_tests 800 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
[ "${SKIP_TESTS:-0}" = 1 ] || step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench_B 600 python3 bench.py --traffic-json $O/pmc_traffic.json
step bench_stream 300 python3 bench.py --workload stream
step bench_stream_host 300 python3 bench.py --workload stream --no-cpu --host-inputs
step bench_B_q2000 400 python3 bench.py --queries 2000
fi
if [ $P2 = 1 ]; then
step bench_stream_ransac 500 python3 bench.py --workload stream --solver RANSAC_DRPM
step bench_A 400 python3 bench.py --workload A
step bench_A_ransac 400 python3 bench.py --workload A --solver RANSAC_DRPM
step bench_E 500 python3 bench.py --workload E
step kt_driver 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_driver -o run -- python3 bench.py --no-cpu --no-host-leg
# the roofline fraction recomputed from the driver command's own kernel trace (tools/trace_frac.py)
f=$(find $O/kt_driver -name '*kernel_trace.csv' | head -1)
python3 tools/trace_frac.py $f $O/kt_driver.out > $O/kt_driver_frac.json && cat $O/kt_driver_frac.json
step kt_single 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_single -o run -- python3 bench.py --no-cpu --no-host-leg --inflight 1 --no-fuse --steps 5 --warmup 1
f=$(find $O/kt_single -name '*kernel_trace.csv' | head -1)
python3 tools/iter_profile.py $f > $O/per_iteration_single_pair.txt && cat $O/per_iteration_single_pair.txt
# the driver's N>1 launch shape at N=1 (torch.distributed.run, RCCL init, max-over-ranks timing)
step dist1 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu
fi
echo done
