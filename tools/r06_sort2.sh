#!/bin/bash
# Round 6: kernel trace of the small pair sort (tile sort / merge passes) in the lone-frame probe
set -u
O=gpurun_out/${OUT:-r06_sort2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/lo_probe.py 10 > $O/kt.out 2> $O/kt.err
echo "kt rc=$?"
f=$(find $O/kt -name '*kernel_stats.csv' | head -1); grep -i "tile_sort\|merge_pass\|merge_tile\|ROCPRIM" $f | cut -c1-200
echo done
