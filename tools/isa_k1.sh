#!/bin/bash
# Device assembly of one K1 instantiation unit (gfx950) for static instruction counts.
# Usage: tools/isa_k1.sh <out.s> [PREC=0] [CMP=0] [source dir=system_identification_amd/csrc]
set -e
out=$1; p=${2:-0}; c=${3:-0}; src=${4:-system_identification_amd/csrc}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -I"$src" -DSYSID_PREC=$p -DSYSID_CMP=$c \
  --cuda-device-only -S -gline-tables-only -o "$out" "$src/sysid_k1_inst.hip"
grep -A40 "\.name:.*k1_regressor_panelILi3ELi18ELi2EdLi0ELi0ELi0" "$out" | grep -E "\.(sgpr|vgpr)_(count|spill_count)" | head -4 || true
