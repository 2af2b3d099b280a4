#!/bin/bash
# Round-4 session 2: the -m gpu suite (3-buffer narrow K2, chunk-major staging), smoke, the narrow-K2 buffer A/B, the
# e2e probe and the record benches.  Stops at the first failure.
set -o pipefail
TAG=${1:-r04_s2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc $rc"; grep -E " passed| failed" $OUT/pytest_gpu.log | tail -2; grep FAILED $OUT/pytest_gpu.log | head
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash tools/lib_ab_bench.sh $TAG/k2_nbuf_ab 3 "--steps 200 --warmup 100 --no-steady-state" system_identification_amd/libsysid.so tools/_libs/k2nb2.so > $OUT/k2_nbuf_ab.txt 2>&1 || { echo "ab failed"; tail $OUT/k2_nbuf_ab.txt; exit 1; }
cat $OUT/k2_nbuf_ab.txt
bash tools/gpu_r04_e2e.sh $TAG/e2e || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo "bench failed"; tail -20 $OUT/bench_driver.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --robot g1_29dof --no-cpu-baseline --no-e2e > $OUT/bench_g1_20k.json 2> $OUT/bench_g1.err || { echo "g1 bench failed"; tail -20 $OUT/bench_g1.err; exit 1; }
timeout -k 10 300 python bench.py --gram-only --no-cpu-baseline > $OUT/bench_spot_gram_only.json 2> $OUT/bench_spot_go.err || { echo "spot gram-only bench failed"; tail -20 $OUT/bench_spot_go.err; exit 1; }
for p in f64 f32 bf16; do
  timeout -k 10 300 python bench.py --robot g1_29dof --samples 1000000 --gram-only --precision $p --no-cpu-baseline --no-e2e --steps 10 --warmup 3 > $OUT/bench_g1_1000000_$p.json 2> $OUT/bench_g1_1000000_$p.err || { echo "g1 1M $p bench failed"; tail -20 $OUT/bench_g1_1000000_$p.err; exit 1; }
done
for f in $OUT/bench*.json; do python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('step_times', {}).get('median_ms'), (d.get('e2e') or {}).get('gram_only'), d['roofline'].get('frac'))"; done
echo S2_DONE
