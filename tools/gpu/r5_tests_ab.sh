#!/bin/bash
# GPU box: the full GPU suite, then a same-box A/B of DDPG_GEMM_M16=0 at C3.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r5_gputests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/r5_gputests.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r5_gputests.log | head -20; tail -30 gpurun_out/r5_gputests.log; exit $rc; }
bash tools/gpu/envab.sh DDPG_GEMM_M16=0 c3 3 gemm_h3 2>&1 | tee gpurun_out/r5_m16_ab_c3.txt
