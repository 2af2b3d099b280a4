#!/bin/bash
# Reduced-precision Gram-only: tests + G1 125k / Spot 200k per precision (+ chunk-size sweep on an EXPERIMENTS build)
set -o pipefail
TAG=${1:-dev}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "precision or gram_only or graph or config5" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log; grep "normwise" $OUT/pytest.log
for p in f64 f32 bf16; do
  timeout -k 10 300 python bench.py --robot g1_29dof --samples 125000 --gram-only --precision $p --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/bench_g1_$p.json 2> $OUT/bench_g1_$p.err || { echo "bench $p failed"; tail -20 $OUT/bench_g1_$p.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_g1_$p.json'));print('g1 $p', d['ms_per_step'], d['kernel_ms'], d['roofline']['kernel'], d['roofline']['frac'])"
done
for mb in 64 128 256 1024; do
  SYSID_LIB=$PWD/tools/_libs/chunk128.so SYSID_GRAM_CHUNK_MB=$mb timeout -k 10 300 python bench.py --robot g1_29dof --samples 125000 --gram-only --precision bf16 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/bench_g1_bf16_c$mb.json 2> $OUT/bench_g1_bf16_c$mb.err || { echo "bench chunk $mb failed"; tail -20 $OUT/bench_g1_bf16_c$mb.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_g1_bf16_c$mb.json'));print('g1 bf16 chunk $mb MB', d['ms_per_step'], d['kernel_ms'])"
done
echo DONE
