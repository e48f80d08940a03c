#!/bin/bash
# GPU box: tests touching the folded Adam + gradient reduction, then same-box A/B (C3, C5)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_graph_pin.py tests/test_gpu_configs.py tests/test_gpu_dp.py tests/test_gpu_parity.py tests/test_gpu_switches.py \
  > gpurun_out/adam_tests.log 2>&1 || { tail -30 gpurun_out/adam_tests.log; exit 1; }
tail -3 gpurun_out/adam_tests.log
bash tools/gpu/ab.sh c3 3
