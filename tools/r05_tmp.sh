set -u
O=gpurun_out/r05l; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_verlet.py tests/test_gpu_bench_path.py tests/test_gpu_frames.py tests/test_gpu_qfuse.py tests/test_gpu_tv.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > $O/tests.out 2>&1 || { echo tests failed; tail -30 $O/tests.out; exit 1; }
tail -1 $O/tests.out
OUT=r05l VARS="base" ROUNDS=3 BENCH_ARGS="--no-host-leg" bash tools/ab_libs.sh || exit 1
OUT=r05l_A VARS="base" ROUNDS=2 BENCH_ARGS="--workload A" bash tools/ab_libs.sh || exit 1
OUT=r05l_s VARS="base" ROUNDS=1 BENCH_ARGS="--workload stream" bash tools/ab_libs.sh || exit 1
timeout -k 10 200 python3 tools/frame_probe.py 40 > $O/probe.txt 2>&1 && head -1 $O/probe.txt
