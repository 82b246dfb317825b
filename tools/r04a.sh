set -u
mkdir -p gpurun_out/r04a
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r04a/gpu_tests.out 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r04a/gpu_tests.out
[ $rc -le 1 ] || exit $rc
OUT=r04a TESTS="tests/test_gpu_parity.py tests/test_gpu_verlet.py tests/test_gpu_bucket.py tests/test_gpu_bench_path.py tests/test_gpu_frames.py tests/test_gpu_batch.py" TEST_ENV="IMLS_LDS_LIST=1" KNOBS="base IMLS_LDS_LIST=1" ROUNDS=2 bash tools/gpu_knobs.sh
timeout -k 10 300 python3 bench.py --no-cpu --host-inputs --steps 8 --latency-pairs 10 > gpurun_out/r04a/bench_B_host.json 2> gpurun_out/r04a/bench_B_host.err
rc=$?; echo "B host rc=$rc"; tail -4 gpurun_out/r04a/bench_B_host.err
