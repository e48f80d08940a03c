#!/bin/bash
# GPU box: isolate a failing bf16 comparison: the same test under the default,
# DDPG_KCOMB=0 (no in-launch K split) and DDPG_TK_LDS=1 (LDS-staged thin_k).
set -o pipefail
mkdir -p gpurun_out
T=tests/test_gpu_switches.py::test_gemm256_switch_bf16
for env in "X=0" "DDPG_KCOMB=0" "DDPG_TK_LDS=1"; do
  env $env timeout -k 10 200 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/iso.log 2>&1
  echo "$env rc=$? $(grep -E 'AssertionError: [0-9.e-]+|passed|failed' gpurun_out/iso.log | head -2 | tr '\n' ' ')"
done
