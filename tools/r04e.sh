set -u
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_verlet.py tests/test_gpu_plane_icp.py tests/test_gpu_projected.py tests/test_gpu_tv.py tests/test_gpu_bench_path.py tests/test_gpu_frames.py tests/test_gpu_bucket.py tests/test_gpu_normals.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.out 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.out
[ $rc -eq 0 ] || exit $rc
OUT=r04e ROUNDS=2 SKIP_DUMP=1 bash tools/gpu_ab.sh
