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
    libtest)  # the parity subset that caught the round's friction-store failure, on each $TEST_LIBS build
      for lib in $TEST_LIBS; do
        n=$(basename $lib .so)
        SYSID_LIB=$PWD/$lib timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "whole_panel or two_streams or determinism or config4_shard" > $OUT/libtest_$n.log 2>&1; rc=$?
        echo "libtest $n rc $rc: $(grep -E ' passed| failed' $OUT/libtest_$n.log | tail -1)"
        [ $rc -eq 0 ] || exit 1  # any failure (a fault reads as a failed test too) ends the session
      done ;;
    pmc)
      bash tools/pmc_ab.sh $OUT/pmc ${PMC_ROBOT:-spot} $PMC_LIBS || exit 1 ;;
    *)
      bash tools/gpu_r06.sh $TAG $step || exit 1 ;;
  esac
done
