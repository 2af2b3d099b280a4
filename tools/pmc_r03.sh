#!/bin/bash
# PMC passes (SQ instruction mix / waits / LDS / MFMA, then FETCH_SIZE and WRITE_SIZE alone) around one workload:
# bash tools/pmc_r03.sh <outdir> <python script and args...>
out=$1; shift
mkdir -p $out
export TMPDIR=/tmp
run() {  # run <tag> <counters...>
  local tag=$1; shift
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" -f csv -d $out/$tag -o run -- python "${ARGS[@]}" > $out/$tag.log 2>&1 || { tail -5 $out/$tag.log; return 1; }
}
ARGS=("$@")
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_MFMA &&
run b SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES &&
run c FETCH_SIZE SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_SMEM &&
run d WRITE_SIZE SQ_INST_CYCLES_VMEM_WR SQ_INSTS_BRANCH &&
python tools/pmc_table.py $out/a $out/b $out/c $out/d > $out/table.txt 2>&1 && rm -rf $out/a $out/b $out/c $out/d && head -200 $out/table.txt
