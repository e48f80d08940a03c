#!/bin/bash
# GPU box: the parity suite, then a same-box A/B of an environment switch
# ($1, e.g. DDPG_GEMM256=0) on a bench config ($2)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/gputests.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "PASS|FAIL|ERROR" gpurun_out/gputests.log | tail -70
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu/envab.sh "$1" "$2"
