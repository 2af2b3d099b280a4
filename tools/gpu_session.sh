#!/bin/bash
# Measurement session for the current tree: the whole -m gpu suite, smoke, the Spot bench at the driver's
# settings (twice) and at its defaults, the G1 20k full-output line, the Spot 20k Gram-only line and
# the G1 125k Gram-only lines.  Every GPU step is time-limited; the script stops at the first failure.
# Usage: bash tools/gpu_session.sh <tag> [quick]   (quick: skip the pytest suite and smoke)
set -o pipefail
TAG=${1:-dev}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "quick" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  grep -E " passed| failed" $OUT/pytest_gpu.log | tail -2
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver_$i.json 2> $OUT/bench_driver.err || { echo "bench failed"; tail -20 $OUT/bench_driver.err; exit 1; }
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --robot g1_29dof --no-cpu-baseline --no-e2e > $OUT/bench_g1_20k.json 2> $OUT/bench_g1.err || { echo "g1 bench failed"; tail -20 $OUT/bench_g1.err; exit 1; }
for p in f64 f32 bf16; do
  timeout -k 10 300 python bench.py --robot g1_29dof --samples 125000 --gram-only --precision $p --no-cpu-baseline --no-e2e --steps 10 --warmup 3 > $OUT/bench_g1_125000_$p.json 2> $OUT/bench_g1_125000_$p.err || { echo "g1 125k $p bench failed"; tail -20 $OUT/bench_g1_125000_$p.err; exit 1; }
done
timeout -k 10 300 python bench.py --gram-only --no-cpu-baseline --no-e2e > $OUT/bench_spot_gram_only.json 2> $OUT/bench_spot_go.err || { echo "spot gram-only bench failed"; tail -20 $OUT/bench_spot_go.err; exit 1; }
for f in $OUT/bench*.json; do python -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); st=d.get('step_times', {})
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d.get('kernel_ms'), st.get('median_ms'), st.get('first_quartile_mean_ms'), st.get('last_quartile_mean_ms'), d['roofline']['frac'])"; done
echo SESSION_DONE
