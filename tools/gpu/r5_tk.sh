#!/bin/bash
# GPU box: thin_k variant G (compile-time plane count, late X-tile wait) through the
# parity / config tests, then same-box A/B of A (HEAD), F, G for C3 and C5
mkdir -p gpurun_out
DDPG_LIB_PATH=tools/ab/libG.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_graph_pin.py > gpurun_out/tk_tests.log 2>&1 \
  || { tail -30 gpurun_out/tk_tests.log; exit 1; }
tail -2 gpurun_out/tk_tests.log
bash tools/gpu/ab.sh c3 3 && bash tools/gpu/ab.sh c5 1
