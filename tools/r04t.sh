set -u
O=gpurun_out/r04t; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 90 env IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/debug/libimls_gpu.so python -u -m pytest "tests/test_gpu_stream.py::test_vlp16_stream_ls[3]" -x -q --timeout 80 --timeout-method thread > $O/t.out 2>&1
rc=$?; echo "rc=$rc"; grep -c "frontier stuck" $O/t.out; grep "frontier stuck" $O/t.out | head -20; tail -5 $O/t.out
