set -u
O=gpurun_out/r04q; mkdir -p $O
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex 'k_knn_qwave_f' --output-format csv --pmc "$@" -d $O/$name -o run -- python3 tools/frame_probe.py 4 > $O/$name.out 2> $O/$name.err
  local rc=$?; echo "pmc $name rc=$rc"; return $rc
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY || exit $?
run sq2 SQ_WAVES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE || exit $?
python3 tools/sq_frame.py k_knn_qwave_f $O/sq1 > $O/sq1.txt; cat $O/sq1.txt
python3 tools/sq_frame.py k_knn_qwave_f $O/sq2 > $O/sq2.txt; cat $O/sq2.txt
