#!/bin/bash
# Round-6 record of the final tree: -m gpu suite, smoke, the bench lines (Spot at the driver's settings and defaults,
# Gram-only, config 4 whole; G1 20k full outputs, 125k bf16, config 5 whole in f64 / f32 / bf16), rocprofv3 kernel
# stats of the driver-settings bench, FETCH_SIZE / WRITE_SIZE passes (pmc_summary.json, read by bench.py for
# roofline.traffic) and SQ counter passes of the Spot headline and the G1 bf16 K1.
# Usage: bash tools/gpu_r06_final.sh [tag] [first step] [stop before step]   (steps: suite bench g1 prof pmc)
set -o pipefail
TAG=${1:-r06_final}
FROM=${2:-suite}
STOP=${3:-none}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
go=0
step() { [ "$1" = "$FROM" ] && go=1; [ "$1" = "$STOP" ] && go=0; [ $go -eq 1 ]; }
if step suite; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc $rc"; grep -E " passed| failed" $OUT/pytest_gpu.log | tail -2; grep FAILED $OUT/pytest_gpu.log | head
  [ $rc -eq 0 ] || exit 1
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
b() {  # b <name> <bench args...>
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -20 $OUT/$name.err; exit 1; }
  python tools/bench_summary.py $OUT/$name.json
}
if step bench; then
  b bench_driver --steps 20 --warmup 5
  b bench_default --no-cpu-baseline --no-e2e
  b bench_spot_gram_only --gram-only --no-cpu-baseline --steps 20 --warmup 5
  b bench_spot_200k --robot spot --total-samples 200000 --no-cpu-baseline --no-e2e --steps 10 --warmup 3
fi
if step g1; then
  b bench_g1_20k --robot g1_29dof --no-cpu-baseline --no-e2e --steps 10 --warmup 3
  b bench_g1_125k_bf16 --robot g1_29dof --samples 125000 --gram-only --precision bf16 --no-cpu-baseline --no-e2e --steps 10 --warmup 3
  for p in bf16 f32 f64; do
    b bench_g1_1000000_$p --robot g1_29dof --samples 1000000 --gram-only --precision $p --no-cpu-baseline --no-e2e --no-steady-state --steps 3 --warmup 1
  done
fi
if step prof; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline --no-e2e --steps 20 --warmup 5 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
  find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \; ; head -6 $OUT/kernel_stats.csv
fi
if step pmc; then
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $OUT/pmc_fetch -o run -- python bench.py --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -20 $OUT/pmc_fetch.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $OUT/pmc_write -o run -- python bench.py --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -20 $OUT/pmc_write.log; exit 1; }
  python tools/pmc_summary.py $OUT $OUT/pmc_summary.json spot 20000 > /dev/null || exit 1
  bash tools/pmc_r03.sh $OUT/pmc_sq bench.py --no-cpu-baseline --no-e2e --no-steady-state --steps 3 --warmup 1 > $OUT/pmc_sq.log 2>&1 || { echo "sq pmc failed"; tail -20 $OUT/pmc_sq.log; exit 1; }
  bash tools/pmc_r03.sh $OUT/pmc_sq_g1 bench.py --robot g1_29dof --samples 125000 --gram-only --precision bf16 --no-cpu-baseline --no-e2e --no-steady-state --steps 3 --warmup 1 > $OUT/pmc_sq_g1.log 2>&1 || { echo "sq pmc g1 failed"; tail -20 $OUT/pmc_sq_g1.log; exit 1; }
fi
echo FINAL_DONE
