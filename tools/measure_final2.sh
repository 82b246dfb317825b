#!/bin/bash
# Round-4 late measurement (profiles/r04_final2): the lone-frame / small-frame paths changed after
# r04_final (fused exact stage, k_fallback_slab, bottom-up + frontier traversal, one-launch frame
# prologue/epilogue); config B's packet kernels did not.  PART=1: GPU suite, smoke, B, stream;
# PART=2: the other legs whose small frames take the changed kernels, and the N=1 torchrun launch.
set -u
O=gpurun_out/${OUT:-final2}
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }
}
if [ "${PART:-1}" = 1 ]; then
[ "${SKIP_TESTS:-0}" = 1 ] || step gpu_tests 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench_B 600 python3 bench.py
step bench_stream 300 python3 bench.py --workload stream
fi
if [ "${PART:-1}" = 2 ]; then
step bench_stream_host 300 python3 bench.py --workload stream --no-cpu --host-inputs
step bench_stream_ransac 400 python3 bench.py --workload stream --no-cpu --solver RANSAC_DRPM
step bench_A 400 python3 bench.py --workload A
step bench_E 500 python3 bench.py --workload E
step bench_B_q2000 400 python3 bench.py --queries 2000
step bench_A_ransac 400 python3 bench.py --workload A --solver RANSAC_DRPM
step bench_B_host 400 python3 bench.py --host-inputs --no-cpu
step dist1 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu
fi
echo done
