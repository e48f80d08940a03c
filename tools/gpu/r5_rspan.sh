#!/bin/bash
# GPU box: same-box A/B of gemm_h3m's fragment-read placement (A = the first
# 18 MFMA gaps, B = spread over 36, C = over 44; tools/mfma_lds_power_bench)
mkdir -p gpurun_out
bash tools/gpu/ab.sh c3 3 && bash tools/gpu/ab.sh c5 2
