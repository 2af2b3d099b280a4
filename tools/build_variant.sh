#!/bin/bash
# Build a library variant with extra defines: bash tools/build_variant.sh <out.so> [-DFOO=1 ...]
out=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude -Isystem_identification_amd/csrc "$@" \
  -o $out system_identification_amd/csrc/sysid_engine.hip system_identification_amd/csrc/sysid_io.cpp \
  system_identification_amd/csrc/sysid_rccl.cpp -lpthread -ldl
