#!/bin/bash
# GPU box: 256x256 GEMM microbench (plain, then fused epilogue), then the
# parity suite and a short bench.  Stops at the first failing GPU step.
mkdir -p gpurun_out
timeout -k 10 120 ./tools/gemmh256_bench > gpurun_out/h256.txt 2>&1 || { echo "h256 rc=$?"; cat gpurun_out/h256.txt; exit 1; }
cat gpurun_out/h256.txt
H2_EPI=1 timeout -k 10 120 ./tools/gemmh256_bench > gpurun_out/h256_epi.txt 2>&1 || { echo "h256 epi rc=$?"; cat gpurun_out/h256_epi.txt; exit 1; }
cat gpurun_out/h256_epi.txt
bash tools/gpu/run_tests_bench.sh
