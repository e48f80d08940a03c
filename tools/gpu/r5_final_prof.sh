#!/bin/bash
# GPU box: the driver's default bench, rocprof evidence for C3 / C5 / C2, and the
# per-rank C3 strong step with its per-call-site kernel list
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu/round_profile.sh || exit $?
mkdir -p gpurun_out/prof_c2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2/trace -o run -- python3 bench.py \
  --config c2 --no-cpu --no-small --steps 50 --warmup 10 > gpurun_out/prof_c2/bench.json \
  2> gpurun_out/prof_c2/bench.err || exit $?
timeout -k 10 300 python -u bench.py --config c3 --per-rank-of 8 --scaling strong --no-cpu --no-small \
  > gpurun_out/per_rank_c3_strong8.json 2> gpurun_out/per_rank_c3_strong8.err || exit $?
echo done
