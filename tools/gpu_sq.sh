#!/bin/bash
# The new packet-size batch test, then two SQ counter passes over the hot kernels in the roofline
# regime (one pair in flight, unfused): wave / instruction / wait counts for DESIGN §5.
set -u
O=gpurun_out/${OUT:-sq}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_frames.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --steps 2 --warmup 1 --no-cpu --inflight 1 --no-fuse --latency-pairs 3"
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --kernel-include-regex 'k_knn_wave|k_finish' --output-format csv \
      --pmc "$@" -d $O/$name -o run -- $B > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "pmc $name rc=$rc"; return $rc
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY || exit $?
run sq2 SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE || exit $?
echo done
