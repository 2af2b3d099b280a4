#!/bin/bash
# Whole -m gpu suite, smoke, the driver-settings bench (with its e2e legs) and kernel times fused / unfused.
set -o pipefail
TAG=${1:-r04_f}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; echo "pytest rc $?"
grep -E "passed|failed|FAILED|ERROR" $OUT/pytest_gpu.log | tail -12
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo "bench failed"; tail -20 $OUT/bench_driver.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_driver.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_ms'], d.get('kernel_ms_fused'), d['step_times']['median_ms'], d.get('steady_state', {}).get('ms_per_step'), d['roofline']['frac'], d.get('e2e'), d.get('cpu_baseline'))"
for i in 1 2; do
  SYSID_LIB=$PWD/tools/_libs/base_r03.so timeout -k 10 120 python tools/quick_time.py spot 20000 2>&1 | grep -v amdgpu.ids | head -2 || exit 1
  timeout -k 10 120 python tools/quick_time.py spot 20000 2>&1 | grep -v amdgpu.ids | head -2 || exit 1
done
echo SESSION_DONE
