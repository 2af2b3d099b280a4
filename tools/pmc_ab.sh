#!/bin/bash
# One SQ pass (instruction mix incl. MFMA) of K1 per library build: bash tools/pmc_ab.sh <outdir> <robot> lib...
# Each pass runs rocprofv3 on tools/k1_only.py (the interpreter straight after `--`), under its own time limit.
out=$1; robot=$2; shift 2
mkdir -p $out
export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename $lib .so)
  SYSID_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES -f csv -d $out/$n -o run -- python tools/k1_only.py $robot 20000 > $out/$n.log 2>&1 || { tail $out/$n.log; exit 1; }
  python tools/pmc_table.py $out/$n > $out/$n.txt 2>&1
  grep -A9 "^k1_regressor_panel" $out/$n.txt
done
