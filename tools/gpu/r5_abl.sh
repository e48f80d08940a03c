#!/bin/bash
# GPU box: gemm_h3 k-loop ablations at M=4096 N=1024 (no epilogue), interleaved
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/h3_abl.txt
for r in 1 2; do
for b in h3_phase_bench h3_phase_bench_NODMA h3_phase_bench_NOREAD h3_phase_bench_NOMFMA h3_phase_bench_NODMA_NOREAD; do
  for K in 2048 1024; do
    echo "== $b K=$K round $r" >> gpurun_out/h3_abl.txt
    timeout -k 10 60 ./tools/$b $K >> gpurun_out/h3_abl.txt 2>&1 || { cat gpurun_out/h3_abl.txt; exit 1; }
  done
done
done
cat gpurun_out/h3_abl.txt
