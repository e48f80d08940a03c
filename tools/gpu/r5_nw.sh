#!/bin/bash
# GPU box: GPU suite, then same-box A/B (tools/ab/libA = before, libB = after) at C3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r5_gputests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/r5_gputests.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r5_gputests.log | head -20; tail -30 gpurun_out/r5_gputests.log; exit $rc; }
bash tools/gpu/ab.sh c3 3
