#!/bin/bash
# GPU box: parity suite, same-box A/B of DDPG_SLOTS_H2D=1 (slot upload) at C2
# and C3, then the host issue cost per step (graph / eager) at C2.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -3 gpurun_out/gputests.log
bash tools/gpu/envab.sh DDPG_SLOTS_H2D=1 c2 > gpurun_out/slots_ab_c2.txt || exit $?
cat gpurun_out/slots_ab_c2.txt
bash tools/gpu/envab.sh DDPG_SLOTS_H2D=1 c3 > gpurun_out/slots_ab_c3.txt || exit $?
cat gpurun_out/slots_ab_c3.txt
timeout -k 10 200 python tools/gpu/host_time.py c2 2>/dev/null | grep -v "^\[bench\]" || exit $?
DDPG_GRAPH=0 timeout -k 10 200 python tools/gpu/host_time.py c2 2>/dev/null | grep -v "^\[bench\]" || exit $?
