#!/bin/bash
# Round-4 session 11: host Gram-only staged-chunk split, 3 chunks (one round + two of whole rounds) vs 2 (one round +
# the rest), Spot 20k, interleaved rounds; then the staged-chunk tests with the 2-split.
set -o pipefail
TAG=${1:-r04_s11}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3; do
  for sp in 3 2; do
    env -u SYSID_STAGE_CHUNKS SYSID_STAGE_SPLIT=$sp SYSID_TRACE_HOST=1 timeout -k 10 120 python tools/e2e_breakdown.py spot 20000 6 > $OUT/e2e_split${sp}_$r.txt 2>&1 || exit 1
    echo "== split $sp round $r"; grep -E "gram_only: python" $OUT/e2e_split${sp}_$r.txt | tail -4 | awk '{print $4}' | tr '\n' ' '; echo; grep -E "flags=8" $OUT/e2e_split${sp}_$r.txt | tail -1
  done
done
SYSID_STAGE_SPLIT=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 120 --timeout-method thread -k "staged_chunks or gram_only_chunked" > $OUT/pytest_staged2.log 2>&1; rc=$?
echo "staged tests (split 2) rc $rc"; grep -E "passed|failed" $OUT/pytest_staged2.log | tail -1
echo S11_DONE
