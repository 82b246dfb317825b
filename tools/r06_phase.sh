#!/bin/bash
# Round 6: phase clocks of the lone frame's k_solve_small (LS) and of the RANSAC hypothesis / DRPM head
# kernels (make debug, copied to csrc/var_dbg/: csrc/debug is not uploaded)
set -u
O=gpurun_out/${OUT:-r06_phase}
mkdir -p $O
export TMPDIR=/tmp
export IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/var_dbg/libimls_gpu.so
timeout -k 10 300 python3 tools/frame_probe.py 20 > $O/frame_probe.out 2> $O/frame_probe.err; echo "frame rc=$?"; cat $O/frame_probe.out
timeout -k 10 300 python3 tools/ransac_probe.py 20 > $O/ransac_probe.out 2> $O/ransac_probe.err; echo "ransac rc=$?"; cat $O/ransac_probe.out
echo done
