#!/bin/bash
# Round-4 session 9: staged chunks on K1 round boundaries (host Gram-only path): staged-chunk tests, then the e2e of
# the default bounds against 1 / 2 equal chunks (tools/e2e_breakdown.py with phase stamps), then the full suite.
set -o pipefail
TAG=${1:-r04_s9}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 120 --timeout-method thread -k "staged_chunks or gram_only_chunked or streamed" > $OUT/pytest_staged.log 2>&1; rc=$?
echo "staged tests rc $rc"; grep -E "passed|failed" $OUT/pytest_staged.log | tail -2; grep FAILED $OUT/pytest_staged.log | head
[ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for ch in default 2 1; do
    if [ $ch = default ]; then env -u SYSID_STAGE_CHUNKS SYSID_TRACE_HOST=1 timeout -k 10 120 python tools/e2e_breakdown.py spot 20000 5 > $OUT/e2e_${ch}_$r.txt 2>&1 || exit 1
    else SYSID_STAGE_CHUNKS=$ch SYSID_TRACE_HOST=1 timeout -k 10 120 python tools/e2e_breakdown.py spot 20000 5 > $OUT/e2e_${ch}_$r.txt 2>&1 || exit 1; fi
    echo "== chunks $ch round $r"; grep -E "gram_only: python" $OUT/e2e_${ch}_$r.txt | tail -3 | tr '\n' ' '; echo; grep -A1 "flags=8" $OUT/e2e_${ch}_$r.txt | tail -2
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc $rc"; grep -E " passed| failed" $OUT/pytest_gpu.log | tail -2; grep FAILED $OUT/pytest_gpu.log | head
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --gram-only --no-cpu-baseline > $OUT/bench_spot_gram_only.json 2> $OUT/bench_spot_go.err || exit 1
python -c "import json; d=json.loads(open('$OUT/bench_spot_gram_only.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['e2e'])"
echo S9_DONE
