#!/bin/bash
# Nullspace graph-replay diagnostic, then fused vs unfused kernel times, the exchange and driver benches, and the
# whole -m gpu suite (no -x: every failure listed).
set -o pipefail
TAG=${1:-r04_c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python tools/dbg_ns_graph.py 4099 2>&1 | grep -v amdgpu.ids || exit 1
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
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo "bench failed"; tail -20 $OUT/bench_driver.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_driver.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['step_times'], d.get('steady_state'), d['roofline'], d.get('e2e'))"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; echo "pytest rc $?"
grep -E "passed|failed|FAILED|ERROR" $OUT/pytest_gpu.log | tail -12
echo SESSION_DONE
