#!/bin/bash
# PMC counters for K1 of a library variant: bash tools/pmc_k1.sh <lib> <outdir> [robot]
lib=$1; out=$2; robot=${3:-spot}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
SYSID_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_WR -f csv -d $out/a -o run -- python tools/k1_only.py $robot 20000 > $out.a.log 2>&1 || exit 1
SYSID_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_WR -f csv -d $out/b -o run -- python tools/k1_only.py $robot 20000 > $out.b.log 2>&1 || exit 1
