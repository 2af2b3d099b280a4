#!/bin/bash
# Round-4 record, part A: the -m gpu suite (with -s: the full-N oracle tests print their times), smoke, the bench at
# the driver's settings and at its defaults, the G1 lines, Spot Gram-only and config 4.  Stops at the first failure.
set -o pipefail
TAG=${1:-r04_final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; echo "pytest rc $?"
grep -E " passed| failed" $OUT/pytest_gpu.log | tail -2; grep FAILED $OUT/pytest_gpu.log | head
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo "bench failed"; tail -20 $OUT/bench_driver.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --robot g1_29dof --no-cpu-baseline --no-e2e > $OUT/bench_g1_20k.json 2> $OUT/bench_g1.err || { echo "g1 bench failed"; tail -20 $OUT/bench_g1.err; exit 1; }
timeout -k 10 300 python bench.py --gram-only --no-cpu-baseline > $OUT/bench_spot_gram_only.json 2> $OUT/bench_spot_go.err || { echo "spot gram-only bench failed"; tail -20 $OUT/bench_spot_go.err; exit 1; }
timeout -k 10 300 python bench.py --robot spot --total-samples 200000 --no-cpu-baseline --no-e2e --steps 10 --warmup 3 > $OUT/bench_spot_200k.json 2> $OUT/bench_spot_200k.err || { echo "spot 200k bench failed"; tail -20 $OUT/bench_spot_200k.err; exit 1; }
for n in 125000 1000000; do
  for p in f64 f32 bf16; do
    timeout -k 10 300 python bench.py --robot g1_29dof --samples $n --gram-only --precision $p --no-cpu-baseline --no-e2e --steps 10 --warmup 3 > $OUT/bench_g1_${n}_$p.json 2> $OUT/bench_g1_${n}_$p.err || { echo "g1 $n $p bench failed"; tail -20 $OUT/bench_g1_${n}_$p.err; exit 1; }
  done
done
for f in $OUT/bench*.json; do python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('step_times', {}).get('median_ms'), (d.get('e2e') or {}).get('gram_only'))"; done
echo FINAL_A_DONE
