#!/bin/bash
# Fused K1 + Gram: its tests, then kernel times fused vs unfused and the old build (tools/_libs/base_r03.so).
set -o pipefail
TAG=${1:-r04_b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_fused.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_fused.log; exit 1; }
grep -E " passed| failed" $OUT/pytest_fused.log | tail -2
for i in 1 2; do
  for lib in tools/_libs/base_r03.so system_identification_amd/libsysid.so; do
    echo "== $lib fused"
    SYSID_LIB=$PWD/$lib timeout -k 10 120 python tools/quick_time.py spot 20000 2>&1 | grep -v amdgpu.ids || exit 1
  done
  echo "== unfused (SYSID_FUSE=0)"
  SYSID_FUSE=0 timeout -k 10 120 python tools/quick_time.py spot 20000 2>&1 | grep -v amdgpu.ids || exit 1
done
for lib in tools/_libs/base_r03.so system_identification_amd/libsysid.so; do
  echo "== gram-only $lib"
  SYSID_LIB=$PWD/$lib timeout -k 10 200 python tools/gram_only_time.py spot 20000 f64 3 2>&1 | grep -v amdgpu.ids || exit 1
  SYSID_LIB=$PWD/$lib timeout -k 10 200 python tools/gram_only_time.py g1_29dof 125000 bf16 2 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --exchange-world1 --no-cpu-baseline --no-e2e --no-steady-state > $OUT/bench_xchg.json 2> $OUT/bench_xchg.err || { echo "xchg bench failed"; tail -20 $OUT/bench_xchg.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_xchg.json').read().strip().splitlines()[-1]); print(d['config']['exchange'], d['config']['exchange_check'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo "bench failed"; tail -20 $OUT/bench_driver.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_driver.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['step_times'], d.get('steady_state'), d['roofline'])"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest -m gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
echo SESSION_DONE
