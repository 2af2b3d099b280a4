#!/bin/bash
# Round-4 last check of the committed tree: -m gpu suite, smoke, the bench at the driver's settings.
set -o pipefail
TAG=${1:-r04_last}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc $rc"; grep -E " passed| failed" $OUT/pytest_gpu.log | tail -2; grep FAILED $OUT/pytest_gpu.log | head
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo "bench failed"; tail -20 $OUT/bench_driver.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_driver.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'], d['steady_state']['ms_per_step'], d['e2e']['gram_only']['ms'], d['cpu_baseline']['value'])"
echo LAST_DONE
