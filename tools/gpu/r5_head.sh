#!/bin/bash
# GPU box: DP tests (in-launch wgrad combine asserted), then same-box A/B of the
# critic-head backward's rows per chunk (A = 64, B = 32, C = 128)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dp.py > gpurun_out/head_tests.log 2>&1 || { tail -40 gpurun_out/head_tests.log; exit 1; }
tail -2 gpurun_out/head_tests.log
bash tools/gpu/ab.sh c3 3 && bash tools/gpu/ab.sh c5 1
