#!/bin/bash
# Round-4 session 4: the -m gpu suite (streamed inputs through host-written flags, part-major DMA), the streamed
# e2e probe over part counts, and the Spot A/B of the K1 input-fetch change (HEAD build vs this tree).
set -o pipefail
TAG=${1:-r04_s4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s --timeout 120 --timeout-method thread -k "streamed" > $OUT/pytest_streamed.log 2>&1; rc=$?
echo "streamed tests rc $rc"; grep -E "PASSED|FAILED|passed|failed" $OUT/pytest_streamed.log | tail -6
[ $rc -eq 0 ] || exit 1
for parts in 2 4 8; do
  SYSID_STREAM_PARTS=$parts SYSID_TRACE_HOST=1 timeout -k 10 60 python tools/stream_probe.py 6 > $OUT/streamed_$parts.txt 2>&1 || exit 1
  echo "== parts $parts"; grep -E "call|flags=8" $OUT/streamed_$parts.txt | tail -4
done
SYSID_STAGE_CHUNKS=2 SYSID_TRACE_HOST=1 timeout -k 10 60 python tools/stream_probe.py 6 > $OUT/chunked_2.txt 2>&1 || exit 1
echo "== chunked 2"; grep -E "call" $OUT/chunked_2.txt | tail -3
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc $rc"; grep -E " passed| failed" $OUT/pytest_gpu.log | tail -2; grep FAILED $OUT/pytest_gpu.log | head
[ $rc -eq 0 ] || exit 1
bash tools/lib_ab_bench.sh $TAG/k1_fetch_ab 3 "--steps 200 --warmup 100 --no-steady-state" system_identification_amd/libsysid.so tools/_libs/base_head.so > $OUT/k1_fetch_ab.txt 2>&1 || { echo "ab failed"; tail $OUT/k1_fetch_ab.txt; exit 1; }
cat $OUT/k1_fetch_ab.txt
echo S4_DONE
