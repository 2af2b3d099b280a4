#!/bin/bash
# A/B variant build from a patched copy of the sources: bash tools/build_patched.sh <out.so> <patch.py> [flags]
# patch.py runs with the copy's csrc directory as its working directory (plain string replacements); the copy
# is built by __graft_entry__.build_library (every translation unit, in parallel).  REUSE=1: start from the tree's
# own objects and recompile only the units whose (patched) sources changed -- only for patches whose extra flags
# matter to the patched units alone.
set -e
out=$(realpath -m $1); patch=$(realpath $2); shift 2
tmp=$(mktemp -d)
cp -r system_identification_amd/csrc $tmp/csrc
force=True
if [ "${REUSE:-0}" = 1 ]; then
  mkdir -p $tmp/obj && sleep 1 && cp -p system_identification_amd/_build/*.o $tmp/obj/ && touch $tmp/obj/*.o && sleep 1
  force=False
fi
(cd $tmp/csrc && python3 $patch)
python3 - "$out" "$tmp" "$force" "$@" <<'PY'
import sys
sys.path.insert(0, ".")
import __graft_entry__ as g
out, tmp, force, extra = sys.argv[1], sys.argv[2], sys.argv[3] == "True", sys.argv[4:]
g.build_library(out=out, csrc=tmp + "/csrc", obj_dir=tmp + "/obj", extra=extra, force=force)
PY
rm -rf $tmp
