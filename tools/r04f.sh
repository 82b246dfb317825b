set -u
O=gpurun_out/${RUNDIR:-r04f}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_single -o run -- python3 bench.py --no-cpu --inflight 1 --no-fuse --steps 5 --warmup 1 --latency-pairs 5 --busy-steps 0 > $O/kt_single.out 2> $O/kt_single.err
rc=$?; echo "kt_single rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/kt_single.err; exit $rc; }
f=$(find $O/kt_single -name '*kernel_trace.csv' | head -1)
python3 tools/iter_profile.py $f > $O/per_iteration_single_pair.txt; cat $O/per_iteration_single_pair.txt
IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/debug/libimls_gpu.so timeout -k 10 300 python3 tools/wave_dump.py 1 2 3 6 12 > $O/wave_dump.txt 2> $O/wave_dump.err
rc=$?; echo "wave_dump rc=$rc"; [ $rc -eq 0 ] || tail -5 $O/wave_dump.err
grep -A1 "== launch" $O/wave_dump.txt
