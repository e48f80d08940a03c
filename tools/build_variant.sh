#!/bin/bash
# Build a tuning variant of libddpg_hip.so with extra compile flags into
# build_variants/lib_<name>.so (load it with DDPG_LIB_PATH=...; experiments only).
#   tools/build_variant.sh <name> [-DFLAG=VALUE ...]
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT/distributed_ddpg_amd/csrc"
mkdir -p "$ROOT/build_variants"
V=$1
shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall \
  -Wno-unused-function -I/opt/rocm/include "$@" gemm.hip step.hip dp.hip replay.hip abi.hip sampler.cpp crc32c.cpp -shared \
  -L/opt/rocm/lib -lrccl -Wl,-soname,libddpg_hip.so -o "$ROOT/build_variants/lib_$V.so"
