#!/bin/bash
# e2e (host entry point) probe: H2D copy shapes, the host phase stamps of the Gram-only call per staging layout and
# chunk count, the streamed form, the new staging test, and a kernel + memory-copy trace.  Stops at the first failure.
set -o pipefail
TAG=${1:-r04_e2e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python tools/h2d_probe.py 71 20000 2 > $OUT/h2d_probe.txt 2>&1 || { echo "h2d probe failed"; tail $OUT/h2d_probe.txt; exit 1; }
cat $OUT/h2d_probe.txt
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "staged_chunks or gram_only_chunked" > $OUT/pytest_staged.log 2>&1 || { echo "staged tests failed"; tail -30 $OUT/pytest_staged.log; exit 1; }
tail -1 $OUT/pytest_staged.log
for lay in rows cm; do
  for ch in 1 2 3 4; do
    SYSID_STAGE_LAYOUT=$lay SYSID_STAGE_CHUNKS=$ch SYSID_TRACE_HOST=1 timeout -k 10 120 python tools/e2e_breakdown.py spot 20000 5 > $OUT/e2e_${lay}_$ch.txt 2>&1 || { echo "breakdown $lay $ch failed"; tail $OUT/e2e_${lay}_$ch.txt; exit 1; }
    echo "== layout $lay chunks $ch"; grep -E "gram_only: python" $OUT/e2e_${lay}_$ch.txt | tail -3; grep -E "flags=8" $OUT/e2e_${lay}_$ch.txt | tail -1; grep -A1 -E "flags=8" $OUT/e2e_${lay}_$ch.txt | grep "chunk stamps" | tail -1
  done
done
for parts in 2 4; do
  SYSID_STREAM_PARTS=$parts SYSID_TRACE_HOST=1 timeout -k 10 120 python tools/e2e_breakdown.py spot 20000 5 > $OUT/e2e_streamed_$parts.txt 2>&1 || { echo "streamed $parts failed"; tail $OUT/e2e_streamed_$parts.txt; exit 1; }
  echo "== streamed $parts"; grep -E "gram_only: python" $OUT/e2e_streamed_$parts.txt | tail -3; grep -E "flags=8" $OUT/e2e_streamed_$parts.txt | tail -1
done
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace -f csv -d $OUT/trace -o run -- python tools/e2e_breakdown.py spot 20000 3 > $OUT/trace.log 2>&1 || { echo "trace failed"; tail $OUT/trace.log; exit 1; }
find $OUT/trace -name "*.csv" | head
echo E2E_DONE
