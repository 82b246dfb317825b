set -u
O=gpurun_out/r04k; mkdir -p $O
OUT=r04k TESTS="tests/test_gpu_parity.py tests/test_gpu_verlet.py tests/test_gpu_bucket.py tests/test_gpu_bench_path.py" TEST_ENV="IMLS_SEED_SKIP=1" KNOBS="base IMLS_SEED_SKIP=1 IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/variant/libimls_gpu.so" ROUNDS=2 bash tools/gpu_knobs.sh
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.out 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $O/gpu_tests.out; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 tools/frame_probe.py 20 > $O/frame_probe.txt 2>&1
rc=$?; echo "probe rc=$rc"; grep -v amdgpu $O/frame_probe.txt
