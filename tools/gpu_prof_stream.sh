#!/bin/bash
# Kernel trace of the fused config-C/D-like stream bench (and the host-time split it logs).
set -u
O=gpurun_out/${OUT:-pst}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --workload stream --no-cpu --steps 5 --warmup 1 ${EXTRA:-} > $O/plain.json 2> $O/plain.err
rc=$?; echo "plain rc=$rc"; tail -3 $O/plain.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --workload stream --no-cpu --steps 5 --warmup 1 ${EXTRA:-} > $O/kt.json 2> $O/kt.err
rc=$?; echo "kt rc=$rc"; exit $rc
