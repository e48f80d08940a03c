#!/bin/bash
# GPU box: the bf16 fused dWa (gemm_h16i epilogue) through the switch / config / DP
# tests, then same-box A/B (A = HEAD, H = this build) for C5 and C3
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_switches.py tests/test_gpu_configs.py tests/test_gpu_dp.py > gpurun_out/nwbf16_tests.log 2>&1 \
  || { tail -40 gpurun_out/nwbf16_tests.log; exit 1; }
tail -2 gpurun_out/nwbf16_tests.log
bash tools/gpu/ab.sh c5 3 && bash tools/gpu/ab.sh c3 2
