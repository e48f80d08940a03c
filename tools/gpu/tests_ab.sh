#!/bin/bash
# GPU box: parity suite, then same-box A/B of tools/ab/lib{A,B}.so at C3 and C5.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -3 gpurun_out/gputests.log
echo "## c3"; bash tools/gpu/ab.sh c3 3 || exit $?
echo "## c5"; bash tools/gpu/ab.sh c5 3 || exit $?
