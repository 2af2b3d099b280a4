#!/bin/bash
# Interleaved e2e A/B of library builds: R rounds of (lib1, lib2, ...) x tools/e2e_time.py, then the median of the
# per-run best and median call times per library.  Usage: bash tools/e2e_ab.sh <tag> <rounds> "<e2e_time args>" lib...
set -o pipefail
TAG=$1; R=$2; ARGS=$3; shift 3
OUT=gpurun_out/$TAG.txt
mkdir -p $(dirname $OUT)
: > $OUT
for r in $(seq 1 $R); do
  for lib in "$@"; do
    SYSID_LIB=$PWD/$lib timeout -k 10 120 python tools/e2e_time.py $ARGS 2>&1 | grep " best " | sed "s|^|$(basename $lib) |" >> $OUT || exit 1
  done
done
python - "$OUT" <<'PY'
import sys, statistics, collections, re
rows = collections.defaultdict(list)
for line in open(sys.argv[1]):
    f = line.split()
    lib = f[0] if len(f) < 5 or f[4] == "gram_only" else f[0] + ":" + f[4]  # per library and output mode
    m = re.search(r"best ([0-9.]+) ms\s+median ([0-9.]+) ms", line)
    rows[lib].append((float(m.group(1)), float(m.group(2))))
for lib, v in rows.items():
    print("%-18s n=%d  best-of-best %.3f  median-of-best %.3f  median-of-median %.3f" % (
        lib, len(v), min(b for b, _ in v), statistics.median(b for b, _ in v), statistics.median(m for _, m in v)))
PY
