set -u
O=gpurun_out/r04i; mkdir -p $O
T="tests/test_gpu_parity.py tests/test_gpu_verlet.py tests/test_gpu_frames.py tests/test_gpu_batch.py tests/test_gpu_stream.py tests/test_gpu_plane_icp.py tests/test_gpu_tv.py tests/test_gpu_ransac.py"
timeout -k 10 700 python -u -m pytest $T -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests_default.out 2>&1
rc=$?; echo "tests default rc=$rc"; tail -3 $O/tests_default.out; [ $rc -eq 0 ] || exit $rc
IMLS_QFINISH=1 timeout -k 10 700 python -u -m pytest $T -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests_qfinish.out 2>&1
rc=$?; echo "tests qfinish rc=$rc"; tail -3 $O/tests_qfinish.out; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/frame_probe.py 20 > $O/frame_probe.txt 2>&1
rc=$?; echo "probe rc=$rc"; grep -v amdgpu $O/frame_probe.txt; [ $rc -eq 0 ] || exit $rc
IMLS_QFINISH=1 timeout -k 10 300 python3 tools/frame_probe.py 20 > $O/frame_probe_qf.txt 2>&1
rc=$?; echo "probe qfinish rc=$rc"; grep -v amdgpu $O/frame_probe_qf.txt
