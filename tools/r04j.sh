set -u
O=gpurun_out/r04j; mkdir -p $O
export TMPDIR=/tmp
for kl in 22 26; do
  IMLS_KL=$kl timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt_kl$kl -o run -- python3 bench.py --no-cpu --inflight 1 --no-fuse --steps 3 --warmup 1 --latency-pairs 3 --busy-steps 0 --no-verify > $O/kt_kl$kl.out 2> $O/kt_kl$kl.err
  rc=$?; echo "kt kl$kl rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/kt_kl$kl.err; exit $rc; }
  f=$(find $O/kt_kl$kl -name '*kernel_trace.csv' | head -1)
  python3 tools/iter_profile.py $f > $O/per_iter_kl$kl.txt; head -2 $O/per_iter_kl$kl.txt
  IMLS_KL=$kl IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/debug/libimls_gpu.so timeout -k 10 300 python3 tools/wave_dump.py 4 6 9 12 > $O/wave_dump_kl$kl.txt 2> $O/wave_dump_kl$kl.err
  rc=$?; echo "wave_dump kl$kl rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/wave_dump_kl$kl.err; exit $rc; }
  grep -A1 "== launch" $O/wave_dump_kl$kl.txt
done
IMLS_QVERLET=1 timeout -k 10 300 python3 tools/frame_probe.py 20 > $O/frame_probe_qv.txt 2>&1
rc=$?; echo "probe qverlet rc=$rc"; grep -v amdgpu $O/frame_probe_qv.txt
IMLS_QVERLET=1 IMLS_QFINISH=1 timeout -k 10 300 python3 tools/frame_probe.py 20 > $O/frame_probe_qvqf.txt 2>&1
rc=$?; echo "probe qverlet+qfinish rc=$rc"; grep -v amdgpu $O/frame_probe_qvqf.txt
