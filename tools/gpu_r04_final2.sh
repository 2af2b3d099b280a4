#!/bin/bash
# Round-4 record of the final tree after the narrow-K2 chunk change (24 rows): -m gpu suite, smoke, the Spot bench
# lines (driver settings, defaults, Gram-only, config 4 whole), rocprofv3 stats, FETCH/WRITE and SQ passes.
set -o pipefail
TAG=${1:-r04_final2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc $rc"; grep -E " passed| failed" $OUT/pytest_gpu.log | tail -2; grep FAILED $OUT/pytest_gpu.log | head
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo "bench failed"; tail -20 $OUT/bench_driver.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --gram-only --no-cpu-baseline > $OUT/bench_spot_gram_only.json 2> $OUT/bench_spot_go.err || { echo "spot gram-only bench failed"; tail -20 $OUT/bench_spot_go.err; exit 1; }
timeout -k 10 300 python bench.py --robot spot --total-samples 200000 --no-cpu-baseline --no-e2e --steps 10 --warmup 3 > $OUT/bench_spot_200k.json 2> $OUT/bench_spot_200k.err || { echo "spot 200k bench failed"; tail -20 $OUT/bench_spot_200k.err; exit 1; }
for f in $OUT/bench*.json; do python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('kernel_ms'), d['roofline'].get('frac'), (d.get('steady_state') or {}).get('ms_per_step'))"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline --no-e2e --steps 20 --warmup 5 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $OUT/pmc_fetch -o run -- python bench.py --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -20 $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $OUT/pmc_write -o run -- python bench.py --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -20 $OUT/pmc_write.log; exit 1; }
python tools/pmc_summary.py $OUT $OUT/pmc_summary.json spot 20000 > /dev/null || exit 1
bash tools/pmc_r03.sh $OUT/pmc_sq bench.py --no-cpu-baseline --no-e2e --no-steady-state --steps 3 --warmup 1 > $OUT/pmc_sq.log 2>&1 || { echo "sq pmc failed"; tail -20 $OUT/pmc_sq.log; exit 1; }
echo FINAL2_DONE
