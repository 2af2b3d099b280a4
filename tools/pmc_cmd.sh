#!/bin/bash
# SQ counter passes (instruction mix, waits, LDS conflicts) around one Python workload:
#   bash tools/pmc_cmd.sh <outdir> <script.py> [args...]
# The interpreter goes straight after rocprofv3's `--`: with --pmc the profiler initialises the GPU in the process
# it starts, so that process must be the program itself (never timeout / env / a shell that execs it).  The time
# limit wraps rocprofv3 from outside.
out=$1; shift
case "$1" in
  *.py) ;;
  *) echo "pmc_cmd.sh: expected a Python script after the output dir, got '$1'" >&2; exit 2 ;;
esac
mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_WR -f csv -d $out/a -o run -- python "$@" > $out/a.log 2>&1 || { tail $out/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_WR -f csv -d $out/b -o run -- python "$@" > $out/b.log 2>&1 || { tail $out/b.log; exit 1; }
python tools/pmc_table.py $out/a $out/b > $out/table.txt 2>&1; head -80 $out/table.txt
