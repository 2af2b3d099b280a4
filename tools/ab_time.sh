#!/bin/bash
# A/B timing of library variants: bash tools/ab_time.sh robot N lib1 lib2 ...
robot=$1; N=$2; shift 2
for lib in "$@"; do
  echo "== $lib"
  SYSID_LIB=$PWD/$lib timeout -k 10 200 python tools/quick_time.py $robot $N || exit 1
done
