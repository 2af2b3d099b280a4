#!/bin/bash
# GPU check: pytest -m gpu (per-test timeout), smoke, default bench.  Usage: bash tools/gpu_check.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-dev}; K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KARG[@]}" > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 200 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo DONE
