#!/bin/bash
# Reduced-precision Gram-only session: tests, G1 125k bench per precision, host e2e probe.
set -o pipefail
TAG=${1:-dev}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "precision or gram_only or graph or config5" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
grep "normwise" $OUT/pytest.log
for p in f64 f32 bf16; do
  timeout -k 10 300 python bench.py --robot g1_29dof --samples 125000 --gram-only --precision $p --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/bench_g1_$p.json 2> $OUT/bench_g1_$p.err || { echo "bench $p failed"; tail -20 $OUT/bench_g1_$p.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_g1_$p.json'));print('$p', d['ms_per_step'], d['kernel_ms'], d['roofline']['kernel'], d['roofline']['frac'])"
done
SYSID_HOST_REGISTER=0 timeout -k 10 200 python tools/e2e_probe.py spot 20000 > $OUT/e2e_reg0.txt 2>&1 || { tail $OUT/e2e_reg0.txt; exit 1; }
SYSID_HOST_REGISTER=1 timeout -k 10 200 python tools/e2e_probe.py spot 20000 > $OUT/e2e_reg1.txt 2>&1 || { tail $OUT/e2e_reg1.txt; exit 1; }
cat $OUT/e2e_reg0.txt $OUT/e2e_reg1.txt
echo DONE
