#!/bin/bash
# GPU box: gemm_h3m (16x16x32) vs gemm_h3 (32x32x16): accuracy check, then
# the K sweep with and without the forward epilogue, kernels interleaved.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/h3_phase_bench 0 > gpurun_out/m16_check.txt 2>&1 || { cat gpurun_out/m16_check.txt; exit 1; }
cat gpurun_out/m16_check.txt
: > gpurun_out/m16_phase.txt
for r in 1 2; do
  for ks in 32 16; do
    echo "== kernel $ks round $r" >> gpurun_out/m16_phase.txt
    timeout -k 10 120 ./tools/h3_phase_bench -1 $ks >> gpurun_out/m16_phase.txt 2>&1 || { cat gpurun_out/m16_phase.txt; exit 1; }
  done
done
cat gpurun_out/m16_phase.txt
