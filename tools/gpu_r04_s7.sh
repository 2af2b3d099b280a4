#!/bin/bash
# Round-4 session 7: the -m gpu suite and the Spot A/B of the quadruped K1's prefetch registers (96 channels, 3 per
# lane, against 192) — this tree vs the previous commit's build.
set -o pipefail
TAG=${1:-r04_s7}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc $rc"; grep -E " passed| failed" $OUT/pytest_gpu.log | tail -2; grep FAILED $OUT/pytest_gpu.log | head
[ $rc -eq 0 ] || exit 1
bash tools/lib_ab_bench.sh $TAG/k1_nxr_ab 3 "--steps 200 --warmup 100 --no-steady-state" system_identification_amd/libsysid.so tools/_libs/base_fetch.so > $OUT/k1_nxr_ab.txt 2>&1 || { echo "ab failed"; tail $OUT/k1_nxr_ab.txt; exit 1; }
cat $OUT/k1_nxr_ab.txt
bash tools/lib_ab_bench.sh $TAG/k1_nxr_ab_go 2 "--gram-only --steps 200 --warmup 100 --no-steady-state" system_identification_amd/libsysid.so tools/_libs/base_fetch.so > $OUT/k1_nxr_ab_go.txt 2>&1 || { echo "ab go failed"; tail $OUT/k1_nxr_ab_go.txt; exit 1; }
cat $OUT/k1_nxr_ab_go.txt
echo S7_DONE
