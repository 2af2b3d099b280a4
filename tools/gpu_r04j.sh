#!/bin/bash
# Stream-flag micro test, streamed host Gram-only inputs (DMA flags) e2e, G1 bf16 K1 phase stamps.
set -o pipefail
export TMPDIR=/tmp
for g in 1 4096; do timeout -k 5 60 ./tools/ubench/stream_flag $g || exit 1; done
for c in 4 2; do
  echo "== SYSID_STREAM_PARTS=$c (DMA flags)"
  SYSID_STREAM_PARTS=$c SYSID_TRACE_HOST=1 timeout -k 10 60 python tools/e2e_breakdown.py spot 20000 4 2>&1 | grep -v amdgpu.ids | grep -E "flags=8|gram_only|Error|error" | tail -4 || exit 1
done
SYSID_LIB=$PWD/tools/_libs/k1_stamps_p2.so timeout -k 5 100 python tools/ab/k1_stamps_run.py g1_29dof 125000 bf16 2>&1 | grep -v amdgpu.ids
echo SESSION_DONE
