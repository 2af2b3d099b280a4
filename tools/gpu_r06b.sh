#!/bin/bash
# Round-6 GPU sessions (second part): bash tools/gpu_r06b.sh <tag> <step>...
#   steps: quick (the quadruped-kernel parity tests), pmc (one SQ pass of K1 per $PMC_LIBS build), and every step
#   of gpu_r06.sh (suite, smoke, bench, gonly, ab: A/B of $AB_LIBS builds, ...)
# Every GPU step runs under its own time limit; the first failing step ends the session.
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    quick)
      timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "spot or solo or quad or golden or determin" > $OUT/pytest_quick.log 2>&1; rc=$?
      echo "quick rc $rc"; grep -E " passed| failed" $OUT/pytest_quick.log | tail -2; grep -E "FAILED|Error" $OUT/pytest_quick.log | head
      [ $rc -eq 0 ] || exit 1 ;;
    pmc)
      bash tools/pmc_ab.sh $OUT/pmc ${PMC_ROBOT:-spot} $PMC_LIBS || exit 1 ;;
    *)
      bash tools/gpu_r06.sh $TAG $step || exit 1 ;;
  esac
done
