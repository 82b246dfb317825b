#!/bin/bash
# PMC counter passes (each its own rocprofv3 run; --pmc never combined with sys/runtime traces).
set -u
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu"
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
i=0
for set in "${PMC_SETS[@]:-}"; do :; done
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --kernel-include-regex "${KREGEX:-k_project_wave}" --output-format csv \
      --pmc "$@" -d gpurun_out/pmc/$name -o run -- $B > gpurun_out/pmc/$name.json 2> gpurun_out/pmc/$name.err
  local rc=$?; echo "pmc $name rc=$rc"; return $rc
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY || exit $?
run sq2 SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE || exit $?
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE || exit $?
echo done
