#!/bin/bash
# Round-3 GPU session: the -m gpu suite (-k selects a subset), smoke, the bench at the driver's settings and
# at the default settings.  Each GPU step time-limited; stops at the first failure.
# Usage: bash tools/gpu_r03.sh <tag> ["<pytest -k expr>"]
set -o pipefail
TAG=${1:-dev}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s "${KARG[@]}" > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
grep -E "passed|failed|Gram|error" $OUT/pytest_gpu.log | tail -20
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo "bench failed"; tail -20 $OUT/bench_driver.err; exit 1; }
cat $OUT/bench_driver.json
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
echo DONE
