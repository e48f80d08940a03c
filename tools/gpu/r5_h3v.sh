#!/bin/bash
# GPU box: gemm_h3m schedule variants (tools/h3v_N), K = 2048 / 4096 no epilogue, interleaved
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/h3v.txt
for r in 1 2; do for v in 0 1 2 3 4; do for K in 2048 4096; do
  echo "== v$v K=$K r$r" >> gpurun_out/h3v.txt
  timeout -k 10 60 ./tools/h3v_$v $K 16 >> gpurun_out/h3v.txt 2>&1 || { cat gpurun_out/h3v.txt; exit 1; }
done; done; done
grep -A1 "==" gpurun_out/h3v.txt | grep -v "^--" | paste - - | awk '{print $2, $3, $4, $7, $8, $(NF-12), $(NF-11), $(NF-8), $(NF-7)}'
