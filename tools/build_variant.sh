#!/bin/bash
# Build a library variant with extra defines: bash tools/build_variant.sh <out.so> [-DFOO=1 ...]
set -e
out=$(realpath -m $1); shift
tmp=$(mktemp -d)
python3 - "$out" "$tmp" "$@" <<'PY'
import sys
sys.path.insert(0, ".")
import __graft_entry__ as g
out, tmp, extra = sys.argv[1], sys.argv[2], sys.argv[3:]
g.build_library(out=out, obj_dir=tmp + "/obj", extra=extra, force=True)
PY
rm -rf $tmp
