#!/bin/bash
# Round-5 GPU session: bash tools/gpu_r05.sh <tag> <step>...   steps: suite smoke bench stamps g1 g1bf16 prof
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
    gonly)
      timeout -k 10 300 python bench.py --gram-only --no-cpu-baseline --steps 20 --warmup 5 > $OUT/bench_spot_gram_only.json 2> $OUT/bench_go.err || { echo "gram-only bench failed"; tail -20 $OUT/bench_go.err; exit 1; }
      python tools/bench_summary.py $OUT/bench_spot_gram_only.json ;;
    stamps)
      SYSID_LIB=$PWD/tools/_libs/stamps0.so timeout -k 10 200 python tools/ab/k1_stamps_run.py spot 20000 f64 > $OUT/stamps_spot.txt 2>&1 || { echo "stamps failed"; tail $OUT/stamps_spot.txt; exit 1; }
      SYSID_LIB=$PWD/tools/_libs/stamps0.so timeout -k 10 200 python tools/ab/k1_stamps_run.py g1_29dof 125000 bf16 > $OUT/stamps_g1_bf16.txt 2>&1 || { echo "stamps g1 failed"; tail $OUT/stamps_g1_bf16.txt; exit 1; }
      cat $OUT/stamps_spot.txt $OUT/stamps_g1_bf16.txt | grep -v amdgpu.ids ;;
    g1bf16)
      timeout -k 10 300 python bench.py --robot g1_29dof --samples 125000 --gram-only --precision bf16 --no-cpu-baseline --no-e2e --steps 10 --warmup 3 > $OUT/bench_g1_125k_bf16.json 2> $OUT/bench_g1.err || { echo "g1 bench failed"; tail -20 $OUT/bench_g1.err; exit 1; }
      python tools/bench_summary.py $OUT/bench_g1_125k_bf16.json ;;
    g1)
      timeout -k 10 300 python bench.py --robot g1_29dof --no-cpu-baseline --no-e2e --steps 10 --warmup 3 > $OUT/bench_g1_20k.json 2> $OUT/bench_g1_20k.err || { echo "g1 20k bench failed"; tail -20 $OUT/bench_g1_20k.err; exit 1; }
      python tools/bench_summary.py $OUT/bench_g1_20k.json ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline --no-e2e --steps 20 --warmup 5 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
      find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \; ; head -8 $OUT/kernel_stats.csv ;;
    e2e)
      : > $OUT/e2e.txt
      for cfg in "" "SYSID_STAGE_SPLIT=2" "SYSID_STAGE_CHUNKS=1" "SYSID_STAGE_CHUNKS=2" "SYSID_STAGE_BOUNDS=4096,12288" "SYSID_STAGE_BOUNDS=4096,8192,16384" "SYSID_STAGE_BOUNDS=2048,8192,14336" "SYSID_STAGE_BOUNDS=6144,14336"; do
        env $cfg timeout -k 10 120 python tools/e2e_time.py spot 20000 10 f32 gram >> $OUT/e2e.txt 2>&1 || { echo "e2e failed ($cfg)"; tail $OUT/e2e.txt; exit 1; }
      done
      timeout -k 10 120 python tools/e2e_time.py spot 20000 10 f64 all >> $OUT/e2e.txt 2>&1 || { echo "e2e f64 failed"; exit 1; }
      timeout -k 10 120 python tools/e2e_time.py spot 20000 5 f32 all >> $OUT/e2e.txt 2>&1 || { echo "e2e f32 failed"; exit 1; }
      SYSID_TRACE_HOST=1 timeout -k 10 120 python tools/e2e_time.py spot 20000 3 f32 gram > $OUT/e2e_trace.txt 2>&1 || { echo "e2e trace failed"; exit 1; }
      grep -v amdgpu.ids $OUT/e2e.txt ;;
    ubench)
      timeout -k 10 120 ./tools/ubench/hbm_rw 2048 > $OUT/hbm_rw.txt 2>&1 && timeout -k 10 120 ./tools/ubench/hbm_rw 512 >> $OUT/hbm_rw.txt 2>&1 || { echo "ubench failed"; cat $OUT/hbm_rw.txt; exit 1; }
      cat $OUT/hbm_rw.txt ;;
    e2etrace)
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -f csv -d $OUT/e2etr -o run -- python tools/e2e_time.py spot 20000 4 f32 gram > $OUT/e2etr.log 2>&1 || { echo "e2e trace failed"; tail $OUT/e2etr.log; exit 1; }
      python tools/trace_timeline.py $(dirname $(find $OUT/e2etr -name "*kernel_trace.csv" | head -1)) 6 30 > $OUT/e2e_timeline.txt; tail -32 $OUT/e2e_timeline.txt ;;
    stamps64)
      SYSID_LIB=$PWD/tools/_libs/stamps0.so timeout -k 10 200 python tools/ab/k1_stamps_run.py g1_29dof 20000 f64 > $OUT/stamps_g1_f64.txt 2>&1 || { echo "stamps failed"; tail $OUT/stamps_g1_f64.txt; exit 1; }
      grep -v amdgpu.ids $OUT/stamps_g1_f64.txt ;;
    e2e2)
      : > $OUT/e2e2.txt
      for cs in 1 2 3; do
        for cfg in "SYSID_STAGE_X=0" "SYSID_STAGE_SPLIT=2" "SYSID_STAGE_BOUNDS=4096,16384" "SYSID_STAGE_BOUNDS=4096,12288,16384"; do
          env SYSID_COPY_STREAMS=$cs $cfg timeout -k 10 120 python tools/e2e_time.py spot 20000 12 f32 gram >> $OUT/e2e2.txt 2>&1 || { echo "e2e failed ($cfg)"; tail $OUT/e2e2.txt; exit 1; }
        done
      done
      grep -v amdgpu.ids $OUT/e2e2.txt ;;
    abk1)
      bash tools/ab_rounds.sh $TAG/abk1 spot 4 tools/_libs/base.so tools/_libs/fric.so tools/_libs/fc.so || exit 1 ;;
    ab)
      bash tools/ab_rounds2.sh $TAG/ab ${AB_ROUNDS:-3} "${AB_WL:-spot_full spot_go g1_full g1_bf16}" $AB_LIBS || exit 1 ;;
    ring)
      for lib in $RING_LIBS; do
        SYSID_LIB=$PWD/$lib timeout -k 10 120 python tools/dbg_ring.py 100001 4 2>&1 | grep -v amdgpu.ids | tee -a $OUT/ring.txt || exit 1
      done ;;
    e2esplit)
      : > $OUT/e2e_split.txt
      for r in $(seq 1 ${E2E_ROUNDS:-3}); do
        for b in ${E2E_BOUNDS:-4096 6144 8192 10240}; do
          SYSID_STAGE_BOUNDS=$b timeout -k 10 120 python tools/e2e_time.py spot 20000 12 f32 gram >> $OUT/e2e_split.txt 2>&1 || { echo "e2e split failed"; tail $OUT/e2e_split.txt; exit 1; }
        done
      done
      grep -v amdgpu.ids $OUT/e2e_split.txt ;;
    e2eenv)
      # host e2e over an environment switch: E2E_VAR, E2E_VALS, E2E_ROUNDS
      : > $OUT/e2e_env.txt
      for r in $(seq 1 ${E2E_ROUNDS:-5}); do
        for v in $E2E_VALS; do
          env $E2E_VAR=$v timeout -k 10 120 python tools/e2e_time.py spot 20000 12 f32 gram 2>&1 | grep -v amdgpu.ids | sed "s/^/$E2E_VAR=$v /" >> $OUT/e2e_env.txt || { echo "e2e env failed"; tail $OUT/e2e_env.txt; exit 1; }
        done
      done
      python - $OUT/e2e_env.txt <<'PY'
import re, sys, statistics, collections
rows = collections.defaultdict(lambda: ([], []))
for l in open(sys.argv[1]):
    m = re.match(r"(\S+) .*best ([\d.]+) ms  median ([\d.]+)", l)
    if m:
        rows[m.group(1)][0].append(float(m.group(2)))
        rows[m.group(1)][1].append(float(m.group(3)))
for k, (b, md) in rows.items():
    print(k, "best", min(b), "median of bests", statistics.median(b), "median of medians", statistics.median(md), len(b))
PY
      ;;
    e2erows)
      : > $OUT/e2e_rows.txt
      for r in 1 2 3; do
        for rows in nullspace projector; do
          timeout -k 10 120 python tools/e2e_time.py spot 20000 12 f32 gram $rows >> $OUT/e2e_rows.txt 2>&1 || { echo "e2e rows failed"; tail $OUT/e2e_rows.txt; exit 1; }
        done
      done
      timeout -k 10 200 python bench.py --gram-only --rows projector --no-cpu-baseline --no-e2e --steps 20 --warmup 5 > $OUT/bench_go_projector.json 2>/dev/null || exit 1
      timeout -k 10 200 python bench.py --gram-only --rows nullspace --no-cpu-baseline --no-e2e --steps 20 --warmup 5 > $OUT/bench_go_nullspace.json 2>/dev/null || exit 1
      grep -v amdgpu.ids $OUT/e2e_rows.txt; python tools/bench_summary.py $OUT/bench_go_projector.json $OUT/bench_go_nullspace.json ;;
    envab)
      # interleaved A/B of one library over an environment switch: ENVAB_VAR, ENVAB_VALS, ENVAB_WL, ENVAB_ROUNDS
      : > $OUT/envab.txt
      for r in $(seq 1 ${ENVAB_ROUNDS:-3}); do
        for v in $ENVAB_VALS; do
          env $ENVAB_VAR=$v timeout -k 10 300 python tools/ab_kernels.py $ENVAB_WL 2>&1 | grep "^AB " | sed "s/libsysid.so/$ENVAB_VAR=$v/" >> $OUT/envab.txt || exit 1
        done
      done
      python - $OUT/envab.txt <<'PY'
import sys, statistics, collections
rows = collections.defaultdict(list)
for line in open(sys.argv[1]):
    p = line.split()
    rows[(p[1], p[2])].append([float(p[4]), float(p[6]), float(p[8])])
for (lib, wl), vs in sorted(rows.items(), key=lambda kv: (kv[0][1], kv[0][0])):
    med = [statistics.median(c) for c in zip(*vs)]
    print("%-10s %-16s n=%d  K1 %.4f  K2 %.4f  K3 %.4f" % (wl, lib, len(vs), *med))
PY
      ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo SESSION_DONE
