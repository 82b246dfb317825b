set -u
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_tv.py tests/test_gpu_type_swap.py tests/test_gpu_verlet.py tests/test_gpu_wire.py tests/test_gpu_bucket.py tests/test_gpu_rccl.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/rest_tests.out 2>&1
rc=$?; echo "rest rc=$rc"; tail -3 $O/rest_tests.out
[ $rc -le 1 ] || exit $rc
OUT=r04b TESTS="tests/test_gpu_parity.py tests/test_gpu_verlet.py tests/test_gpu_bucket.py tests/test_gpu_bench_path.py tests/test_gpu_frames.py tests/test_gpu_batch.py" TEST_ENV="IMLS_LDS_LIST=1" KNOBS="base IMLS_LDS_LIST=1" ROUNDS=2 bash tools/gpu_knobs.sh
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --workload stream --no-cpu --latency-pairs 30 > $O/bench_stream.json 2> $O/bench_stream.err
rc=$?; echo "stream rc=$rc"; tail -3 $O/bench_stream.err
