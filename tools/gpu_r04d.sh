#!/bin/bash
# Bisect the graph-replay failures of test_no_state_carried_in_the_workspace by test subset.
set -o pipefail
export TMPDIR=/tmp
run() { timeout -k 10 300 python -u -m pytest "$@" -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | grep -E "passed|failed|FAILED" | tail -4; }
echo "== g1 alone"; run "tests/test_gpu_fused.py::test_no_state_carried_in_the_workspace[g1_29dof-auto]"
echo "== nullspace alone"; run "tests/test_gpu_fused.py::test_no_state_carried_in_the_workspace[spot-nullspace]"
echo "== no_state x3"; run tests/test_gpu_fused.py -k no_state
echo "== fused file"; run tests/test_gpu_fused.py
echo "== parity then fused"; run tests/test_gpu_parity.py tests/test_gpu_fused.py
echo SESSION_DONE
