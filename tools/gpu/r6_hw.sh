#!/bin/bash
# hw GEMM microbenchmark: plain output, then the dX epilogue
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/hw_bench > gpurun_out/hw.txt 2>&1 || { echo "hw rc=$?"; cat gpurun_out/hw.txt; exit 1; }
cat gpurun_out/hw.txt
HW_EPI=1 timeout -k 10 120 ./tools/hw_bench dx > gpurun_out/hw_epi.txt 2>&1 || { echo "hw epi rc=$?"; cat gpurun_out/hw_epi.txt; exit 1; }
cat gpurun_out/hw_epi.txt
