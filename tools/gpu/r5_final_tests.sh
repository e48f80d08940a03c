#!/bin/bash
# GPU box: the whole GPU suite on the in-tree build, then smoke()
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/gputests_final.log 2>&1 || { tail -40 gpurun_out/gputests_final.log; exit 1; }
tail -3 gpurun_out/gputests_final.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -3
