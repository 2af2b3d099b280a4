#!/bin/bash
# Graph replay after a 0xFF workspace: the memset-zeroed counters (tools/_libs/memset_ctr.so) against the kernel-
# zeroed ones (the product), then the fused test file.
set -o pipefail
export TMPDIR=/tmp
for lib in tools/_libs/memset_ctr.so system_identification_amd/libsysid.so; do
  echo "== $lib"
  SYSID_LIB=$PWD/$lib timeout -k 10 120 python tools/dbg_ns_graph.py spot nullspace 2>&1 | grep -v amdgpu.ids || exit 1
  SYSID_LIB=$PWD/$lib timeout -k 10 120 python tools/dbg_ns_graph.py g1_29dof auto 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | grep -E "passed|failed|FAILED" | tail -6
echo SESSION_DONE
