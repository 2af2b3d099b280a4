#!/bin/bash
# Full round-end GPU session: tools/gpu_configs.sh (suite, smoke, bench, G1 lines), then the rocprofv3 kernel
# stats of the default bench and the FETCH_SIZE / WRITE_SIZE PMC passes (each its own run).
# Usage: bash tools/gpu_final.sh <tag>
set -o pipefail
TAG=${1:-dev}
OUT=gpurun_out/$TAG
bash tools/gpu_configs.sh $TAG || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline --steps 20 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $OUT/pmc_fetch -o run -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -20 $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $OUT/pmc_write -o run -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -20 $OUT/pmc_write.log; exit 1; }
find $OUT -name "*.csv" | head -20
echo FINAL_DONE
