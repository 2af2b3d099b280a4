#!/bin/bash
# Interleaved bench.py A/B of library builds: bash tools/lib_ab_bench.sh <tag> <rounds> "<bench args>" lib1 lib2 ...
# (each lib through SYSID_LIB; prints ms per step and kernel ms per run, then the median step per lib)
set -o pipefail
TAG=$1; R=$2; ARGS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in $(seq 1 $R); do
  for lib in "$@"; do
    n=$(basename $lib .so)
    SYSID_LIB=$PWD/$lib timeout -k 10 200 python bench.py $ARGS --no-cpu-baseline --no-e2e > $OUT/${n}_$r.json 2>> $OUT/err.txt || exit 1
  done
done
python - $OUT "$@" <<'PY'
import json, sys, statistics, os
out, libs = sys.argv[1], sys.argv[2:]
for lib in libs:
    n = os.path.basename(lib)[:-3]
    runs = []
    for f in sorted(os.listdir(out)):
        if f.startswith(n + "_") and f.endswith(".json"):
            d = json.loads(open(os.path.join(out, f)).read().strip().splitlines()[-1])
            runs.append((d["ms_per_step"], d["kernel_ms"]))
    for ms, k in runs:
        print(n, ms, {a: b for a, b in k.items() if a != "samples_timed"})
    print("==", n, "median ms per step", statistics.median(r[0] for r in runs))
PY
