#!/bin/bash
# Round 6: per-wave records of the packet traversal per ICP iteration (debug build var_dbg), and one
# SQ pass of the product vs the v_readlane broadcast scan (var_oldbc), one pair in flight.
set -u
O=gpurun_out/${OUT:-r06_wtrace}
mkdir -p $O
export TMPDIR=/tmp
IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/var_dbg/libimls_gpu.so timeout -k 10 300 python3 tools/wave_dump.py 1 2 3 4 6 10 20 > $O/waves.txt 2> $O/waves.err
echo "waves rc=$?"; grep "==\|mean" $O/waves.txt
for v in product oldbc; do
  if [ $v = product ]; then unset IMLS_LIB_PATH; else export IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/var_$v/libimls_gpu.so; fi
  timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex 'k_knn_wave|k_finish' --output-format csv \
    --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY \
    -d $O/sq_$v -o run -- python3 bench.py --no-host-leg --steps 2 --warmup 1 --no-cpu --inflight 1 --no-fuse --latency-pairs 2 > $O/sq_$v.out 2> $O/sq_$v.err
  echo "sq $v rc=$?"
done
unset IMLS_LIB_PATH
echo done
