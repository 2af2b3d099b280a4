#!/bin/bash
# A/B variant build from a patched copy of the sources: bash tools/build_patched.sh <out.so> <patch.py> [flags]
# patch.py runs with the copy's csrc directory as its working directory (plain string replacements).
set -e
out=$(realpath -m $1); patch=$(realpath $2); shift 2
tmp=$(mktemp -d)
cp -r system_identification_amd/csrc $tmp/csrc
(cd $tmp/csrc && python3 $patch)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude -I$tmp/csrc "$@" \
  -o $out $tmp/csrc/sysid_engine.hip $tmp/csrc/sysid_io.cpp $tmp/csrc/sysid_rccl.cpp -lpthread -ldl
rm -rf $tmp
