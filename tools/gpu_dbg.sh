#!/bin/bash
# K12 NaN diagnostic: the per-wave record build, then the unfused path on the same protocol.
set -o pipefail
export TMPDIR=/tmp
echo "== k12_diag"
SYSID_LIB=$PWD/tools/_libs/k12_diag.so timeout -k 10 150 python tools/dbg_k12_nan.py 4099 20000 2>&1 | grep -v amdgpu.ids || exit 1
echo "== unfused (SYSID_FUSE=0)"
SYSID_FUSE=0 timeout -k 10 120 python tools/dbg_k12_nan.py 4099 20000 2>&1 | grep -v amdgpu.ids || exit 1
