#!/bin/bash
# GPU box: the actor head finished in the forward GEMM's epilogue -- the whole GPU suite
# on the in-tree build, then same-box A/B (A = HEAD, F = it), C3 and C5
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/fin_tests.log 2>&1 || { tail -40 gpurun_out/fin_tests.log; exit 1; }
tail -2 gpurun_out/fin_tests.log
bash tools/gpu/ab.sh c3 3 && bash tools/gpu/ab.sh c5 1
