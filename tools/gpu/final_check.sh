#!/bin/bash
# GPU box: parity suite, the driver's default bench, a same-box A/B of the
# small-path issue policy at C2, then rocprof evidence for C3 / C5 / C2.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -3 gpurun_out/gputests.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
head -c 700 gpurun_out/bench_default.json; echo
bash tools/gpu/envab.sh DDPG_GRAPH_AUTO=0 c2 > gpurun_out/auto_ab_c2.txt || exit $?
cat gpurun_out/auto_ab_c2.txt
bash tools/gpu/profile.sh c3 > gpurun_out/prof_c3.log 2>&1 || exit $?
bash tools/gpu/profile.sh c5 > gpurun_out/prof_c5.log 2>&1 || exit $?
mkdir -p gpurun_out/prof_c2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2/trace -o run -- python3 bench.py \
  --config c2 --no-cpu --no-small --steps 50 --warmup 10 > gpurun_out/prof_c2/bench.json \
  2> gpurun_out/prof_c2/bench.err || exit $?
DB=$(find gpurun_out/prof_c2/trace -name '*results.db' | head -1)
python3 profiles/summarize.py $DB > gpurun_out/prof_c2/kernels_c2.txt
echo done
