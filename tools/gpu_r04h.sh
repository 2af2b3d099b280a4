#!/bin/bash
# Host Gram-only e2e vs the number of staged chunks, then the host / parity GPU tests.
set -o pipefail
export TMPDIR=/tmp
for c in 1 2 4 8; do
  echo "== SYSID_STAGE_CHUNKS=$c"
  SYSID_STAGE_CHUNKS=$c SYSID_TRACE_HOST=1 timeout -k 10 120 python tools/e2e_breakdown.py spot 20000 4 2>&1 | grep -v amdgpu.ids | grep -E "flags=8|gram_only" | tail -4 || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_host_api.py tests/test_gpu_configs.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | grep -E "passed|failed|FAILED" | tail -4
echo SESSION_DONE
