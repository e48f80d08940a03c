#!/bin/bash
# GPU box: parity suite, then same-box A/B of the thin_k row-tile walk
# (DDPG_TK_RPB=1 = one row tile per block) at C3 and C5, then a C3 kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -3 gpurun_out/gputests.log
bash tools/gpu/envab.sh DDPG_TK_RPB=1 c3 > gpurun_out/tk_ab_c3.txt || exit $?
cat gpurun_out/tk_ab_c3.txt
bash tools/gpu/envab.sh DDPG_TK_RPB=1 c5 > gpurun_out/tk_ab_c5.txt || exit $?
cat gpurun_out/tk_ab_c5.txt
mkdir -p gpurun_out/tk_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tk_trace/trace -o run -- python3 bench.py \
  --config c3 --no-cpu --no-small --steps 20 --warmup 5 > gpurun_out/tk_trace/bench.json \
  2> gpurun_out/tk_trace/bench.err || exit $?
DB=$(find gpurun_out/tk_trace/trace -name '*results.db' | head -1)
python3 profiles/summarize.py $DB > gpurun_out/tk_trace/kernels_c3.txt
grep thin_k gpurun_out/tk_trace/kernels_c3.txt
