set -u
O=gpurun_out/r04g; mkdir -p $O
OUT=r04g TESTS="tests/test_gpu_parity.py tests/test_gpu_verlet.py tests/test_gpu_bench_path.py" TEST_ENV="IMLS_LEAF_PAIR=1" KNOBS="base IMLS_LEAF_PAIR=1" ROUNDS=2 bash tools/gpu_knobs.sh
rc=$?; [ $rc -le 1 ] || exit $rc
RUNDIR=r04g bash tools/r04f.sh
rc=$?; [ $rc -le 1 ] || exit $rc
IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/debug/libimls_gpu.so timeout -k 10 300 python3 tools/frame_probe.py 20 > gpurun_out/r04g/frame_probe_debug.txt 2>&1
rc=$?; echo "frame_probe debug rc=$rc"; [ $rc -le 1 ] || exit $rc; cat gpurun_out/r04g/frame_probe_debug.txt | grep -v amdgpu.ids
timeout -k 10 300 python3 tools/frame_probe.py 20 > gpurun_out/r04g/frame_probe.txt 2>&1
echo "frame_probe rc=$?"; cat gpurun_out/r04g/frame_probe.txt | grep -v amdgpu.ids
