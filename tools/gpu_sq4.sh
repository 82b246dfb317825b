#!/bin/bash
# SQ counters of the projection kernels in the regime the headline bench runs (config B, 4 pairs in
# flight as 4 launch sequences: the batched k_knn_wave_b / k_finish_b), for the product defaults and
# for each extra knob set in KNOBS (e.g. "IMLS_LDS_LIST=0"): two --pmc passes per variant (8 SQ
# counters at most per pass), summarised per dispatch and per wave by tools/sq_summary.py.
set -u
O=gpurun_out/${OUT:-sq4}
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu --latency-pairs 2 --busy-steps 0 --no-verify"
run() {  # name, env, counters...
  local name=$1 envs=$2; shift 2
  timeout -s KILL 240 env $envs rocprofv3 --kernel-trace --kernel-include-regex 'k_knn_wave_b|k_finish_b' --output-format csv \
      --pmc "$@" -d $O/$name -o run -- $B > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "pmc $name rc=$rc"; return $rc
}
for k in base ${KNOBS:-}; do
  e=$k; [ "$k" = base ] && e="IMLS_NOTHING=0"
  n=$(echo "$k" | tr '=/+' '___')
  run ${n}_sq1 "$e" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY || exit $?
  run ${n}_sq2 "$e" SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE || exit $?
  python3 tools/sq_summary.py $O/${n}_sq1 $O/${n}_sq2 > $O/${n}_summary.txt && cat $O/${n}_summary.txt
done
echo done
