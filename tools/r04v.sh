set -u
O=gpurun_out/r04v; mkdir -p $O
export TMPDIR=/tmp
V=planetary-lidar-odometry_amd/csrc/variant/libimls_gpu.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_qfuse.py tests/test_gpu_verlet.py tests/test_gpu_bucket.py tests/test_gpu_parity.py tests/test_gpu_stream.py -x -q --timeout 200 --timeout-method thread > $O/tests.out 2>&1
rc=$?; echo "tests rc=$rc"; tail -30 $O/tests.out | grep -v "^\.\.\.\." | tail -25; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for k in base IMLS_QEXACT=0; do
    e=$k; [ $k = base ] && e=IMLS_NOTHING=0
    timeout -k 10 100 env $e python3 tools/frame_probe.py 30 > $O/probe_${r}_${k//[=\/]/_}.txt 2>&1 || { echo "probe $k failed"; exit 1; }
    echo "r$r $k: $(head -1 $O/probe_${r}_${k//[=\/]/_}.txt)"
  done
done
timeout -k 10 100 env IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/debug/libimls_gpu.so python3 tools/frame_probe.py 20 > $O/probe_debug.txt 2>&1; echo "debug probe rc=$?"; tail -1 $O/probe_debug.txt
OUT=r04v/stream KNOBS="base IMLS_QEXACT=0" ROUNDS=2 STEPS=6 LAT=20 BENCH_ARGS="--workload stream" bash tools/gpu_knobs.sh
