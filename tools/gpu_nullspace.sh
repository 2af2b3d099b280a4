#!/bin/bash
# Nullspace Gram-only rows: the GPU suite, then the bench's Gram-only step with nullspace vs projector rows
# (Spot 20k f64, G1 125k f64 / bf16) and the default bench.  Usage: bash tools/gpu_nullspace.sh <tag> [-k expr]
set -o pipefail
TAG=${1:-dev}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$2" ]; then KARG=(-k "$2"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s "${KARG[@]}" > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
grep -E "passed|failed|nullspace" $OUT/pytest_gpu.log | tail -8
B="timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --gram-only"
for rows in nullspace projector; do
  $B --robot spot --samples 20000 --rows $rows > $OUT/spot_f64_$rows.json 2> $OUT/err.txt || { tail $OUT/err.txt; exit 1; }
  $B --robot g1_29dof --samples 125000 --rows $rows > $OUT/g1_f64_$rows.json 2> $OUT/err.txt || { tail $OUT/err.txt; exit 1; }
  $B --robot g1_29dof --samples 125000 --precision bf16 --rows $rows > $OUT/g1_bf16_$rows.json 2> $OUT/err.txt || { tail $OUT/err.txt; exit 1; }
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > $OUT/bench_default.json 2> $OUT/err.txt || { tail $OUT/err.txt; exit 1; }
python - <<'PY'
import json, glob, os
out = os.environ.get("OUT_DIR")
PY
for f in $OUT/*.json; do python -c "
import json,sys; d=json.load(open('$f')); k=d['kernel_ms']
print('%-28s ms/step %.4f  K1 %.4f K2 %.4f K3 %.4f  roof %.3f' % ('$(basename $f)', d['ms_per_step'], k['K1_regressor_panel'], k['K2_gram_syrk'], k['K3_gram_reduce'], d['roofline']['frac']))"; done
echo DONE
