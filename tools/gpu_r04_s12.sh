#!/bin/bash
# Round-4 session 12: quadruped K1 with one row-load register set (tools/ab/k1_single_rowbuf.py) vs the product.
set -o pipefail
TAG=${1:-r04_s12}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/lib_ab_bench.sh $TAG/k1_rowbuf_ab 3 "--steps 200 --warmup 100 --no-steady-state" system_identification_amd/libsysid.so tools/_libs/k1_rowbuf1.so > $OUT/k1_rowbuf_ab.txt 2>&1 || { echo "ab failed"; tail $OUT/k1_rowbuf_ab.txt; exit 1; }
cat $OUT/k1_rowbuf_ab.txt
echo S12_DONE
