#!/bin/bash
# SQ counter passes (instruction mix, waits, LDS conflicts) around any command: bash tools/pmc_cmd.sh <outdir> <cmd...>
out=$1; shift
mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_WR -f csv -d $out/a -o run -- "$@" > $out/a.log 2>&1 || { tail $out/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_WR -f csv -d $out/b -o run -- "$@" > $out/b.log 2>&1 || { tail $out/b.log; exit 1; }
python tools/pmc_table.py $out/a $out/b > $out/table.txt 2>&1; cat $out/table.txt | head -80
