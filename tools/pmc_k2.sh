#!/bin/bash
# PMC counters for the Gram kernel of a library variant: bash tools/pmc_k2.sh <lib> <outdir> [robot] [N]
lib=$1; out=$2; robot=${3:-spot}; n=${4:-20000}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
SYSID_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -f csv -d $out/a -o run -- python tools/k1_only.py $robot $n gram > $out.a.log 2>&1 || exit 1
SYSID_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM -f csv -d $out/b -o run -- python tools/k1_only.py $robot $n gram > $out.b.log 2>&1 || exit 1
