set -u
OUT=r04c TESTS="tests/test_gpu_parity.py tests/test_gpu_verlet.py tests/test_gpu_bucket.py tests/test_gpu_bench_path.py tests/test_gpu_frames.py tests/test_gpu_batch.py" KNOBS="base IMLS_LDS_LIST=0 IMLS_KL=24 IMLS_SEED_KEYS=1 IMLS_BCAST_LOCK=1 IMLS_PACKET_BATCH=1" ROUNDS=2 bash tools/gpu_knobs.sh
