set -u
O=gpurun_out/r04r; mkdir -p $O
timeout -k 10 180 env IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/debug/libimls_gpu.so python3 tools/qwave_dump.py > $O/qwave_dump.txt 2>&1
rc=$?; echo "dump rc=$rc"; cat $O/qwave_dump.txt | tail -40
