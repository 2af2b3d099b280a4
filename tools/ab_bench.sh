#!/bin/bash
# Interleaved A/B of the whole bench step: R rounds of (lib1, lib2, ...), bench.py defaults (Spot 20k, 200 steps
# after 100 warmup), then the median ms_per_step per lib.  Usage: bash tools/ab_bench.sh <tag> <rounds> lib1 lib2 ...
set -o pipefail
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG.txt
mkdir -p gpurun_out
: > $OUT
for r in $(seq 1 $R); do
  for lib in "$@"; do
    v=$(SYSID_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernel_ms']['K1_regressor_panel'], d['kernel_ms']['K2_gram_syrk'])") || exit 1
    echo "$lib $v" >> $OUT
  done
done
python - "$OUT" <<'PY'
import sys, statistics
rows = {}
for line in open(sys.argv[1]):
    f = line.split()
    rows.setdefault(f[0], []).append([float(x) for x in f[1:]])
for lib, vs in rows.items():
    med = [statistics.median(c) for c in zip(*vs)]
    print("%-28s n=%d median ms_per_step %.4f  K1 %.4f  K2 %.4f" % (lib, len(vs), *med))
PY
