#!/bin/bash
# Test-only variant of the library whose RCCL calls go to tools/rccl_shm.cpp
# (N rank processes on ONE GPU through /dev/shm; tests/test_gpu_dp_shm.py).
# Reuses the product objects of distributed_ddpg_amd/csrc (make first) and
# links the stand-in instead of librccl: tools/shm/libddpg_shm.so.
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
CSRC="$ROOT/distributed_ddpg_amd/csrc"
make -C "$CSRC" -j4 >/dev/null
mkdir -p "$ROOT/tools/shm"
/opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -Wall -I/opt/rocm/include -c "$ROOT/tools/rccl_shm.cpp" \
  -o "$ROOT/tools/shm/rccl_shm.o"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$CSRC"/build/*.o "$ROOT/tools/shm/rccl_shm.o" \
  -shared -lrt -Wl,-soname,libddpg_hip.so -o "$ROOT/tools/shm/libddpg_shm.so"
