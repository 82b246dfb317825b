set -u
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plane_icp.py tests/test_gpu_projected.py tests/test_gpu_ransac.py tests/test_gpu_tv.py tests/test_gpu_normals.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.out 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.out
[ $rc -eq 0 ] || exit $rc
OUT=r04d/sq KNOBS="IMLS_LDS_LIST=0" bash tools/gpu_sq4.sh
