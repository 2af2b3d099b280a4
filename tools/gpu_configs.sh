#!/bin/bash
# GPU session: full -m gpu suite, smoke, default bench, then the G1 bench lines (20k full outputs; the 1M-job
# share of 125k samples Gram-only in f64 / f32 / bf16).  Usage: bash tools/gpu_configs.sh <tag>
set -o pipefail
TAG=${1:-dev}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 200 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 python bench.py --robot g1_29dof --no-cpu-baseline --no-e2e > $OUT/bench_g1_20k.json 2> $OUT/bench_g1.err || { echo "g1 bench failed"; tail -20 $OUT/bench_g1.err; exit 1; }
for p in f64 f32 bf16; do
  timeout -k 10 300 python bench.py --robot g1_29dof --samples 125000 --gram-only --precision $p --no-cpu-baseline --no-e2e --steps 10 --warmup 3 > $OUT/bench_g1_125k_$p.json 2> $OUT/bench_g1_$p.err || { echo "g1 $p bench failed"; tail -20 $OUT/bench_g1_$p.err; exit 1; }
done
python - <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/bench*.json") if len(sys.argv) > 1 else []):
    pass
PY
for f in $OUT/bench_g1*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['kernel_ms'])"; done
echo DONE
