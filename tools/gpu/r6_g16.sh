#!/bin/bash
# GPU box: the 16-row gather -- its bitwise switch test, then same-box A/B
# (A = default gather16; B = DDPG_GATHER16=0) at C3
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu tests/test_gpu_switches.py -k "GATHER16 or SLOTS_H2D" -x -q --timeout 300 --timeout-method thread > gpurun_out/g16_tests.log 2>&1 || { tail -30 gpurun_out/g16_tests.log; exit 1; }
tail -2 gpurun_out/g16_tests.log
bash tools/gpu/envab.sh DDPG_GATHER16=0 c3 2 gather && bash tools/gpu/envab.sh DDPG_GATHER16=0 c5 3 gather || exit $?
