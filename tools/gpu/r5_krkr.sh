#!/bin/bash
# GPU box: weight gradients on gemm_h3m (16x16x32, KR x KR) -- config / parity / graph-pin
# tests on that build, then same-box A/B (A = HEAD, K = it) for C3
mkdir -p gpurun_out
DDPG_LIB_PATH=tools/ab/libK.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  -m gpu tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_graph_pin.py > gpurun_out/krkr_tests.log 2>&1 \
  || { tail -40 gpurun_out/krkr_tests.log; exit 1; }
tail -2 gpurun_out/krkr_tests.log
bash tools/gpu/ab.sh c3 3
