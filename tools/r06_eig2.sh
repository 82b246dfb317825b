set -u
mkdir -p gpurun_out/r06_eig2
IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/var_dbg/libimls_gpu.so timeout -k 10 300 python3 tools/ransac_probe.py 10 > gpurun_out/r06_eig2/phase.out 2> gpurun_out/r06_eig2/phase.err; echo "phase rc=$?"; cat gpurun_out/r06_eig2/phase.out
