set -u
O=gpurun_out/r04u; mkdir -p $O
export TMPDIR=/tmp
V=planetary-lidar-odometry_amd/csrc/variant/libimls_gpu.so
for r in 1 2; do
  for k in base IMLS_FRONTIER=0; do
    e=$k; [ $k = base ] && e=IMLS_NOTHING=0
    timeout -k 10 100 env $e python3 tools/frame_probe.py 30 > $O/probe_${r}_${k//[=\/]/_}.txt 2>&1 || { echo "probe $k failed rc=$?"; exit 1; }
    echo "r$r $k: $(head -1 $O/probe_${r}_${k//[=\/]/_}.txt)"
  done
done
timeout -k 10 100 env IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/debug/libimls_gpu.so python3 tools/qwave_dump.py > $O/qwave_dump.txt 2>&1
rc=$?; echo "dump rc=$rc"; grep -v "late wave" $O/qwave_dump.txt | grep -v "^ *$" | head -30
