#!/bin/bash
# GPU box: dW3 fused into the dz2 thin_k launch -- the switch / config / DP / parity
# tests, then same-box A/B (A = HEAD, W = this build) for C3 and C5
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_switches.py tests/test_gpu_configs.py tests/test_gpu_dp.py tests/test_gpu_parity.py \
  tests/test_gpu_graph_pin.py > gpurun_out/w3_tests.log 2>&1 || { tail -40 gpurun_out/w3_tests.log; exit 1; }
tail -2 gpurun_out/w3_tests.log
bash tools/gpu/ab.sh c3 3 && bash tools/gpu/ab.sh c5 2
