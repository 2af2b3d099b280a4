#!/bin/bash
# G1 Gram-only 125k per precision + G1 20k full, per library: bash tools/g1_precisions.sh lib1 lib2 ...
set -o pipefail
for lib in "$@"; do
  echo "== $lib"
  SYSID_LIB=$PWD/$lib timeout -k 10 100 python tools/quick_time.py g1_29dof 20000 2>&1 | grep "per kernel" || exit 1
  for p in f64 f32 bf16; do
    SYSID_LIB=$PWD/$lib timeout -k 10 200 python bench.py --robot g1_29dof --samples 125000 --gram-only --precision $p --no-cpu-baseline --no-e2e --steps 10 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('  125k gram-only', '$p', d['ms_per_step'], 'ms', d['kernel_ms'])" || exit 1
  done
done
echo DONE
