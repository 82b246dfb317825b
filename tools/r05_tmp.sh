set -u
O=gpurun_out/r05k; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_verlet.py tests/test_gpu_bench_path.py tests/test_gpu_frames.py tests/test_gpu_qfuse.py -x -q --timeout 120 --timeout-method thread > $O/tests.out 2>&1 || { echo tests failed; tail -30 $O/tests.out; exit 1; }
tail -1 $O/tests.out
OUT=r05k VARS="base" ROUNDS=3 BENCH_ARGS="--no-host-leg" bash tools/ab_libs.sh || exit 1
OUT=r05k_s VARS="base" ROUNDS=1 BENCH_ARGS="--workload stream" bash tools/ab_libs.sh || exit 1
