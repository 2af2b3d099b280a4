#!/bin/bash
# A/B variant build from a patched copy of the sources: bash tools/build_patched.sh <out.so> <patch.py> [flags]
# patch.py runs with the copy's csrc directory as its working directory (plain string replacements); the copy
# is built by __graft_entry__.build_library (every translation unit, in parallel).
set -e
out=$(realpath -m $1); patch=$(realpath $2); shift 2
tmp=$(mktemp -d)
cp -r system_identification_amd/csrc $tmp/csrc
(cd $tmp/csrc && python3 $patch)
python3 - "$out" "$tmp" "$@" <<'PY'
import sys
sys.path.insert(0, ".")
import __graft_entry__ as g
out, tmp, extra = sys.argv[1], sys.argv[2], sys.argv[3:]
g.build_library(out=out, csrc=tmp + "/csrc", obj_dir=tmp + "/obj", extra=extra, force=True)
PY
rm -rf $tmp
