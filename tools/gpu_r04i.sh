#!/bin/bash
# Streamed host Gram-only inputs: e2e by parts per shard (0 = the chunked staging), then the host / parity / configs
# GPU tests.
set -o pipefail
export TMPDIR=/tmp
for c in 4 0 2 8; do
  echo "== SYSID_STREAM_PARTS=$c"
  SYSID_STREAM_PARTS=$c SYSID_STAGE_CHUNKS=2 SYSID_TRACE_HOST=1 timeout -k 10 60 python tools/e2e_breakdown.py spot 20000 4 2>&1 | grep -v amdgpu.ids | grep -E "flags=8|gram_only|Error|error" | tail -4 || exit 1
done
SYSID_TRACE_HOST=1 timeout -k 10 60 python tools/e2e_breakdown.py g1_29dof 20000 3 2>&1 | grep -v amdgpu.ids | grep -E "flags=8|gram_only|Error|error" | tail -3 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_host_api.py tests/test_gpu_configs.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | grep -E "passed|failed|FAILED" | tail -4
echo SESSION_DONE
