#!/bin/bash
# Interleaved A/B kernel timing: R rounds of (lib1, lib2, ...) on one robot, then the median per lib.
# Usage: bash tools/ab_rounds.sh <tag> <robot> <rounds> lib1 lib2 ...
set -o pipefail
TAG=$1; ROBOT=$2; R=$3; shift 3
OUT=gpurun_out/$TAG.txt
mkdir -p gpurun_out
: > $OUT
for r in $(seq 1 $R); do
  for lib in "$@"; do
    echo "== $lib" >> $OUT
    SYSID_LIB=$PWD/$lib timeout -k 10 120 python tools/quick_time.py $ROBOT 20000 2>&1 | grep "ms per kernel" >> $OUT || exit 1
  done
done
python - "$OUT" <<'PY'
import re, sys, statistics
rows = {}
lib = None
for line in open(sys.argv[1]):
    if line.startswith("== "):
        lib = line.split()[1]
    elif "ms per kernel" in line:
        v = [float(x) for x in re.findall(r"'([\d.]+)'", line)]
        rows.setdefault(lib, []).append(v)
for lib, vs in rows.items():
    med = [statistics.median(c) for c in zip(*vs)]
    print("%-28s n=%d median [K1, K2, K3] = [%s] total %.4f" % (lib, len(vs), ", ".join("%.4f" % x for x in med), sum(med)))
PY
