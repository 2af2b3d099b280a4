#!/bin/bash
# One GPU session: tests, smoke, bench, rocprof kernel stats + PMC passes.  Each GPU step is time-limited
# and the chain stops at the first failure.  Usage: bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-dev}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -20 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 200 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline --steps 20 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $OUT/pmc_fetch -o run -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -20 $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $OUT/pmc_write -o run -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -20 $OUT/pmc_write.log; exit 1; }
find $OUT -name "*.csv" | head -20
echo DONE
