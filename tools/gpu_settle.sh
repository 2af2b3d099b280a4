#!/bin/bash
# Bench at the driver's settings with and without the clock settle, twice each, interleaved.
set -o pipefail
OUT=gpurun_out/${1:-settle}
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --settle-ms 0 --no-cpu-baseline > $OUT/drv_nosettle_$i.json 2> $OUT/err_$i.txt || exit 1
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/drv_settle_$i.json 2>> $OUT/err_$i.txt || exit 1
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > $OUT/default.json 2>> $OUT/err_1.txt || exit 1
for f in $OUT/*.json; do python -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['step_times']['first_quartile_mean_ms'], d['step_times']['last_quartile_mean_ms'], d['kernel_ms'], d.get('settle'))"; done
