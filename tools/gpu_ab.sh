#!/bin/bash
# A/B kernel timing of library variants + optional pytest subset on the default build.
# Usage: bash tools/gpu_ab.sh <tag> "<pytest -k expr or empty>" lib1 lib2 ...
set -o pipefail
TAG=$1; K=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
for lib in "$@"; do
  for robot in spot g1_29dof; do
    echo "== $lib $robot"
    SYSID_LIB=$PWD/$lib timeout -k 10 120 python tools/quick_time.py $robot 20000 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
echo DONE
