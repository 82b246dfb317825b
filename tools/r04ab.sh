set -u
O=gpurun_out/r04ab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_frame -o run -- python3 tools/frame_probe.py 10 > $O/kt_frame.out 2> $O/kt_frame.err
rc=$?; echo "kt_frame rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $O/kt_frame -name '*kernel_trace.csv' | head -1)
python3 tools/iter_profile_frame.py $f > $O/per_iteration_frame.txt; cat $O/per_iteration_frame.txt
f=$(find $O/kt_frame -name '*kernel_stats.csv' | head -1); cp $f $O/kernel_stats_frame.csv; head -12 $O/kernel_stats_frame.csv | cut -d, -f1-4 | cut -c1-120
