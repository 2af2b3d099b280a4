#!/bin/bash
# e2e breakdown of the host entry point (C phases + Python wall), then the chunked Gram-only test.
set -o pipefail
export TMPDIR=/tmp
SYSID_TRACE_HOST=1 timeout -k 10 120 python tools/e2e_breakdown.py spot 20000 5 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_host_api.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | grep -E "passed|failed|FAILED" | tail -4
echo SESSION_DONE
