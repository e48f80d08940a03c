#!/bin/bash
# GPU box: the parity suite, then same-box A/Bs of DDPG_GEMM_H3=0 at C5 and C3
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/gputests.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "FAIL|ERROR|passed|failed" gpurun_out/gputests.log | tail -10
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "== C5"; bash tools/gpu/envab.sh DDPG_GEMM_H3=0 c5 || exit $?
echo "== C3"; bash tools/gpu/envab.sh DDPG_GEMM_H3=0 c3
