set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03_i
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "snake14" > gpurun_out/r03_i/snake_tests.log 2>&1 || { tail -40 gpurun_out/r03_i/snake_tests.log; exit 1; }
grep -i "snake\|passed\|failed" gpurun_out/r03_i/snake_tests.log | tail -8
for p in f64 f32 bf16; do
  timeout -k 10 300 python bench.py --robot g1_29dof --samples 1000000 --gram-only --precision $p --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/r03_i/bench_g1_1m_$p.json 2> gpurun_out/r03_i/bench_g1_1m_$p.err || { tail -5 gpurun_out/r03_i/bench_g1_1m_$p.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/r03_i/bench_g1_1m_$p.json').read().strip().splitlines()[-1]); print('$p', d['value'], d['ms_per_step'], d.get('kernel_ms'))"
done
