#!/bin/bash
# Round-4 first session: suite + smoke on the tree, the bench with and without the clock settle, and K1 at one
# wave per SIMD (tools/ab/k1_occ1.py) against the default occupancy.
set -o pipefail
TAG=${1:-r04_a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
grep -E " passed| failed" $OUT/pytest_gpu.log | tail -2
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo "bench failed"; tail -20 $OUT/bench_driver.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --settle-ms 0 --no-cpu-baseline > $OUT/bench_nosettle.json 2> $OUT/bench_nosettle.err || { echo "bench failed"; tail -20 $OUT/bench_nosettle.err; exit 1; }
for lib in system_identification_amd/libsysid.so tools/_libs/k1_occ1.so system_identification_amd/libsysid.so tools/_libs/k1_occ1.so; do
  for robot in spot g1_29dof; do
    echo "== $lib $robot"
    SYSID_LIB=$PWD/$lib timeout -k 10 120 python tools/quick_time.py $robot 20000 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
for f in $OUT/bench*.json; do python -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); st=d.get('step_times', {})
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d.get('kernel_ms'), st.get('median_ms'), st.get('first_quartile_mean_ms'), st.get('last_quartile_mean_ms'), d['roofline']['frac'])"; done
echo SESSION_DONE
