#!/bin/bash
# GPU box: thin_k register-epilogue kernel -- switch / parity tests, then a
# same-box A/B against the LDS-staged kernel at C3 and C5.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_switches.py tests/test_gpu_dp.py -x -v \
  --timeout 120 --timeout-method thread -k "kernel_switch or placement or skinny or slots or kcomb or small_m" \
  > gpurun_out/tk_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -25 gpurun_out/tk_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu/envab.sh DDPG_TK_LDS=1 c3 2 thin_k 2>&1 | tee gpurun_out/tk_ab_c3.txt || exit $?
bash tools/gpu/envab.sh DDPG_TK_LDS=1 c5 2 thin_k 2>&1 | tee gpurun_out/tk_ab_c5.txt
