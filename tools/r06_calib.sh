#!/bin/bash
# Round 6: (1) FETCH_SIZE / WRITE_SIZE calibration of the 16-B gather patterns (tools/calib), two
# separate --pmc passes; (2) kernel trace of the shipped solver's lone frame (RANSAC -> DRPM);
# (3) SQ counters of the rejected quad exact stage (var_quad) at 4 pairs in flight.
set -u
O=gpurun_out/${OUT:-r06_calib}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- tools/calib/gather_cal > $O/fetch.out 2> $O/fetch.err
echo "fetch rc=$?"
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- tools/calib/gather_cal > $O/write.out 2> $O/write.err
echo "write rc=$?"
python3 tools/calib/gather_cal.py $O > $O/cal.txt 2>&1; echo "cal rc=$?"; cat $O/cal.txt
timeout -k 10 300 python3 tools/ransac_probe.py 30 > $O/ransac_probe.out 2> $O/ransac_probe.err; echo "ransac probe rc=$?"; cat $O/ransac_probe.out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_ransac -o run -- python3 tools/ransac_probe.py 10 > $O/kt_ransac.out 2> $O/kt_ransac.err
echo "kt ransac rc=$?"
OUT=${OUT:-r06_calib}/sq4_quad KNOBS="IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/var_quad/libimls_gpu.so" bash tools/gpu_sq4.sh > $O/sq4_quad.log 2>&1; echo "sq4 rc=$?"
echo done
