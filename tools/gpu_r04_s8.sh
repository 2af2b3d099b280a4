#!/bin/bash
# Round-4 session 8: narrow K2 rows per staged chunk (Spot: the product, then variant builds), interleaved A/B.
set -o pipefail
TAG=${1:-r04_s8}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/lib_ab_bench.sh $TAG/k2_kc_ab 3 "--steps 200 --warmup 100 --no-steady-state" system_identification_amd/libsysid.so tools/_libs/k2kc28.so tools/_libs/k2kc20.so > $OUT/k2_kc_ab.txt 2>&1 || { echo "ab failed"; tail $OUT/k2_kc_ab.txt; exit 1; }
cat $OUT/k2_kc_ab.txt
echo S8_DONE
