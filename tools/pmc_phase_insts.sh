#!/bin/bash
# K1 instruction counts per library variant (phase-skip builds): bash tools/pmc_phase_insts.sh <tag> lib1 lib2 ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for lib in "$@"; do
  n=$(basename $lib .so)
  SYSID_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY -f csv -d $OUT/$n -o run -- python tools/k1_only.py spot 20000 > $OUT/$n.log 2>&1 || { echo "$n failed"; tail -5 $OUT/$n.log; exit 1; }
  python tools/pmc_table.py $OUT/$n > $OUT/$n.txt 2>&1
  echo "== $n"; grep -A6 k1_regressor $OUT/$n.txt | head -7
done
echo DONE
