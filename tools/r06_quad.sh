#!/bin/bash
# Round 6: the quad exact stage (product) — its parity / batch / fallback tests, then a same-box A/B
# against the one-lane k_finish (var_oldfinish) and the quad kernel with a 24-entry list (var_kl24).
set -u
O=gpurun_out/${OUT:-r06_quad}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_verlet.py tests/test_gpu_plane_icp.py \
    tests/test_gpu_tv.py tests/test_gpu_bench_path.py tests/test_gpu_qfuse.py tests/test_gpu_frames.py tests/test_gpu_batch.py \
    tests/test_gpu_projected.py tests/test_gpu_normals.py tests/test_gpu_bucket.py \
    -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
OUT=${OUT:-r06_quad}/ab VARS="${VARS:-oldfinish kl24}" ROUNDS=${ROUNDS:-2} bash tools/ab_libs.sh
