#!/bin/bash
# Round 6: lone RANSAC frame — DRPM head slabs in LDS, both hypothesis chunks under one selection.
set -u
O=gpurun_out/${OUT:-r06_ransac5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_ransac.py tests/test_gpu_stream.py tests/test_gpu_frames.py \
    tests/test_gpu_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/var_dbg/libimls_gpu.so timeout -k 10 300 python3 tools/ransac_probe.py 20 > $O/phase.out 2> $O/phase.err; echo "phase rc=$?"; cat $O/phase.out
timeout -k 10 300 python3 tools/ransac_probe.py 30 > $O/ransac_probe.out 2> $O/ransac_probe.err; echo "probe rc=$?"; cat $O/ransac_probe.out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_ransac -o run -- python3 tools/ransac_probe.py 10 > $O/kt_ransac.out 2> $O/kt_ransac.err
echo "kt rc=$?"
echo done
