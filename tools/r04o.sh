set -u
O=gpurun_out/r04o; mkdir -p $O
export TMPDIR=/tmp
V=planetary-lidar-odometry_amd/csrc/variant/libimls_gpu.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_qfuse.py tests/test_gpu_verlet.py tests/test_gpu_stream.py -x -q --timeout 200 --timeout-method thread > $O/tests.out 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.out; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for k in base IMLS_QFUSE=0 IMLS_LIB_PATH=$V; do
    e=$k; [ $k = base ] && e=IMLS_NOTHING=0
    timeout -k 10 120 env $e python3 tools/frame_probe.py 30 > $O/probe_${r}_${k//[=\/]/_}.txt 2>&1 || exit 1
    echo "r$r $k: $(head -1 $O/probe_${r}_${k//[=\/]/_}.txt)"
  done
done
timeout -k 10 120 env IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/debug/libimls_gpu.so python3 tools/frame_probe.py 20 > $O/probe_debug.txt 2>&1; echo "debug probe rc=$?"; tail -1 $O/probe_debug.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_frame -o run -- python3 tools/frame_probe.py 10 > $O/kt_frame.out 2> $O/kt_frame.err
rc=$?; echo "kt_frame rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $O/kt_frame -name '*kernel_trace.csv' | head -1)
python3 tools/iter_profile_frame.py $f > $O/per_iteration_frame.txt; cat $O/per_iteration_frame.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.out 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.out
