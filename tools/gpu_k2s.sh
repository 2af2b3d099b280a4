#!/bin/bash
# Structured-Gram session: the Spot/solo12 GPU parity subset, then the bench at the driver's settings with and
# without the clock settle, and the structured vs dense K2 (SYSID_K2_STRUCT=0) at steady state.
set -o pipefail
OUT=gpurun_out/${1:-k2s}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s \
  -k "structured or spot or solo12 or degenerate or determinism or ill_conditioned" > $OUT/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
grep -E "passed|failed|structured" $OUT/pytest_gpu.log | tail -8
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --settle-ms 0 --no-cpu-baseline > $OUT/drv_nosettle_$i.json 2>> $OUT/err.txt || exit 1
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/drv_settle_$i.json 2>> $OUT/err.txt || exit 1
done
for i in 1 2; do
  SYSID_K2_STRUCT=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > $OUT/dense_$i.json 2>> $OUT/err.txt || exit 1
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > $OUT/struct_$i.json 2>> $OUT/err.txt || exit 1
done
for f in $OUT/*.json; do python -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); st=d['step_times']
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], st['first_quartile_mean_ms'], st['last_quartile_mean_ms'], d['kernel_ms'], d.get('settle'), d['roofline']['frac'])"; done
