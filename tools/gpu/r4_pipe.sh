#!/bin/bash
# GPU box: pipe-kernel tests, then same-box A/B (A = default, B = DDPG_TK_PIPE=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_switches.py -x -q --timeout 200 --timeout-method thread -k "pipe or placement" > gpurun_out/pipe_tests.log 2>&1
rc=$?; tail -1 gpurun_out/pipe_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pipe_tests.log | head -20; tail -20 gpurun_out/pipe_tests.log; exit $rc; }
echo "== C3"; bash tools/gpu/envab.sh DDPG_TK_PIPE=1 c3 3 thin_k 2>&1 | tee gpurun_out/pipe_ab_c3.txt || exit 1
echo "== C5"; bash tools/gpu/envab.sh DDPG_TK_PIPE=1 c5 2 thin_k 2>&1 | tee gpurun_out/pipe_ab_c5.txt
