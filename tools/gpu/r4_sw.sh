#!/bin/bash
# GPU box: same-box A/B of existing switches at C5 / C3 on the final build
set -o pipefail
mkdir -p gpurun_out
echo "== GEMM256=1 c5"; bash tools/gpu/envab.sh DDPG_GEMM256=1 c5 2 gemm 2>&1 | tee gpurun_out/g256_ab_c5.txt || exit 1
echo "== PAR=1 c5"; bash tools/gpu/envab.sh DDPG_PAR=1 c5 2 2>&1 | tee gpurun_out/par_ab_c5.txt || exit 1
echo "== PAR=1 c3"; bash tools/gpu/envab.sh DDPG_PAR=1 c3 2 2>&1 | tee gpurun_out/par_ab_c3.txt
