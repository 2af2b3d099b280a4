#!/bin/bash
# G1 125k Gram-only step of one precision per library: bash tools/g1_prec_ab.sh <f64|f32|bf16> lib1 lib2 ...
set -o pipefail
P=$1; shift
for lib in "$@"; do
  SYSID_LIB=$PWD/$lib timeout -k 10 200 python bench.py --robot g1_29dof --samples 125000 --gram-only --precision $P --no-cpu-baseline --no-e2e --steps 10 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('%-32s 125k gram-only $P' % '$lib', d['ms_per_step'], 'ms', d['kernel_ms'])" || exit 1
done
