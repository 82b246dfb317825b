set -u
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.out 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $O/gpu_tests.out; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/frame_probe.py 20 > $O/frame_probe.txt 2>&1
rc=$?; echo "probe rc=$rc"; grep -v amdgpu $O/frame_probe.txt; [ $rc -eq 0 ] || exit $rc
OUT=r04k KNOBS="base" ROUNDS=1 bash tools/gpu_knobs.sh
