#!/bin/bash
# Round-4 record, part B: rocprofv3 kernel stats of the driver-settings bench, its FETCH_SIZE / WRITE_SIZE passes,
# and the SQ counter passes of the Spot headline and of G1 125k bf16 Gram-only (each pass its own run).
set -o pipefail
TAG=${1:-r04_final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline --no-e2e --steps 20 --warmup 5 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $OUT/pmc_fetch -o run -- python bench.py --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -20 $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $OUT/pmc_write -o run -- python bench.py --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -20 $OUT/pmc_write.log; exit 1; }
python tools/pmc_summary.py $OUT $OUT/pmc_summary.json spot 20000 > /dev/null && find $OUT -name "*stats.csv" | head
bash tools/pmc_r03.sh $OUT/pmc_sq bench.py --no-cpu-baseline --no-e2e --no-steady-state --steps 3 --warmup 1 > $OUT/pmc_sq.log 2>&1 || { echo "sq pmc failed"; tail -20 $OUT/pmc_sq.log; exit 1; }
bash tools/pmc_r03.sh $OUT/pmc_sq_g1_bf16 bench.py --robot g1_29dof --samples 125000 --gram-only --precision bf16 --no-cpu-baseline --no-e2e --no-steady-state --steps 3 --warmup 1 > $OUT/pmc_sq_g1.log 2>&1 || { echo "sq pmc g1 failed"; tail -20 $OUT/pmc_sq_g1.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo "bench failed"; tail -20 $OUT/bench_driver.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_driver.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'], d['steady_state']['ms_per_step'], d['e2e']['gram_only']['ms'])"
echo FINAL_B_DONE
