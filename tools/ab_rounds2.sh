#!/bin/bash
# Interleaved A/B of library builds over the ab_kernels.py workloads: R rounds of (lib1, lib2, ...), then the median
# per (lib, workload, kernel).  Usage: bash tools/ab_rounds2.sh <tag> <rounds> "<workloads>" lib1 lib2 ...
set -o pipefail
TAG=$1; R=$2; WLS=$3; shift 3
OUT=gpurun_out/$TAG.txt
mkdir -p $(dirname $OUT)
: > $OUT
for r in $(seq 1 $R); do
  for lib in "$@"; do
    SYSID_LIB=$PWD/$lib timeout -k 10 300 python tools/ab_kernels.py $WLS 2>&1 | grep "^AB " >> $OUT || exit 1
  done
done
python - "$OUT" <<'PY'
import sys, statistics, collections
rows = collections.defaultdict(list)
for line in open(sys.argv[1]):
    p = line.split()
    rows[(p[1], p[2])].append([float(p[4]), float(p[6]), float(p[8])])
for (lib, wl), vs in sorted(rows.items(), key=lambda kv: (kv[0][1], kv[0][0])):
    med = [statistics.median(c) for c in zip(*vs)]
    print("%-12s %-10s n=%d  K1 %.4f  K2 %.4f  K3 %.4f  total %.4f" % (wl, lib, len(vs), *med, sum(med)))
PY
