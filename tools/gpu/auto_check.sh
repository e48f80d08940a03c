#!/bin/bash
# GPU box: parity suite, then same-box A/B of DDPG_GRAPH_AUTO=0 (always the
# graph) at C2, C3, C5.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -3 gpurun_out/gputests.log
for c in c2 c3 c5; do
  bash tools/gpu/envab.sh DDPG_GRAPH_AUTO=0 $c > gpurun_out/auto_ab_$c.txt || exit $?
  echo "## $c"; cat gpurun_out/auto_ab_$c.txt
done
