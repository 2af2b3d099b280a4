#!/bin/bash
# Round-6 GPU session: bash tools/gpu_r06.sh <tag> <step>...   steps: suite smoke bench gonly g1 g1bf16 prof ab e2e
# Every GPU step runs under its own time limit; the first failing step ends the session.
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    suite)
      timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
      echo "pytest rc $rc"; grep -E " passed| failed" $OUT/pytest_gpu.log | tail -2; grep FAILED $OUT/pytest_gpu.log | head
      [ $rc -eq 0 ] || exit 1 ;;
    smoke)
      timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
      tail -1 $OUT/smoke.log ;;
    bench)
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo "bench failed"; tail -20 $OUT/bench_driver.err; exit 1; }
      python tools/bench_summary.py $OUT/bench_driver.json ;;
    bdef)
      timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
      python tools/bench_summary.py $OUT/bench_default.json ;;
    gonly)
      timeout -k 10 300 python bench.py --gram-only --no-cpu-baseline --steps 20 --warmup 5 > $OUT/bench_spot_gram_only.json 2> $OUT/bench_go.err || { echo "gram-only bench failed"; tail -20 $OUT/bench_go.err; exit 1; }
      python tools/bench_summary.py $OUT/bench_spot_gram_only.json ;;
    g1bf16)
      timeout -k 10 300 python bench.py --robot g1_29dof --samples 125000 --gram-only --precision bf16 --no-cpu-baseline --no-e2e --steps 10 --warmup 3 > $OUT/bench_g1_125k_bf16.json 2> $OUT/bench_g1.err || { echo "g1 bench failed"; tail -20 $OUT/bench_g1.err; exit 1; }
      python tools/bench_summary.py $OUT/bench_g1_125k_bf16.json ;;
    g1)
      timeout -k 10 300 python bench.py --robot g1_29dof --no-cpu-baseline --no-e2e --steps 10 --warmup 3 > $OUT/bench_g1_20k.json 2> $OUT/bench_g1_20k.err || { echo "g1 20k bench failed"; tail -20 $OUT/bench_g1_20k.err; exit 1; }
      python tools/bench_summary.py $OUT/bench_g1_20k.json ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline --no-e2e --steps 20 --warmup 5 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
      find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \; ; head -8 $OUT/kernel_stats.csv ;;
    ab)
      bash tools/ab_rounds2.sh $TAG/ab ${AB_ROUNDS:-3} "${AB_WL:-spot_full spot_go g1_full g1_bf16}" $AB_LIBS || exit 1 ;;
    e2e)
      : > $OUT/e2e.txt
      for r in $(seq 1 ${E2E_ROUNDS:-3}); do
        timeout -k 10 120 python tools/e2e_time.py spot 20000 12 f32 gram >> $OUT/e2e.txt 2>&1 || { echo "e2e failed"; tail $OUT/e2e.txt; exit 1; }
      done
      grep -v amdgpu.ids $OUT/e2e.txt ;;
    e2eab)
      bash tools/e2e_ab.sh $TAG/e2eab ${E2E_ROUNDS:-4} "spot 20000 12 f32 gram" $AB_LIBS || exit 1 ;;
    e2etrace)
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -f csv -d $OUT/e2etr -o run -- python tools/e2e_time.py spot 20000 4 f32 gram > $OUT/e2etr.log 2>&1 || { echo "e2e trace failed"; tail $OUT/e2etr.log; exit 1; }
      python tools/trace_timeline.py $(dirname $(find $OUT/e2etr -name "*kernel_trace.csv" | head -1)) 6 30 > $OUT/e2e_timeline.txt; tail -32 $OUT/e2e_timeline.txt
      SYSID_TRACE_HOST=1 timeout -k 10 120 python tools/e2e_time.py spot 20000 4 f32 gram > $OUT/e2e_host_trace.txt 2>&1 || { echo "host trace failed"; exit 1; }
      grep -v amdgpu.ids $OUT/e2e_host_trace.txt | tail -8 ;;
    *)
      echo "unknown step $step"; exit 1 ;;
  esac
done
