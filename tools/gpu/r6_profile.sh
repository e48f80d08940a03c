#!/bin/bash
# GPU box: the driver's default bench command, then rocprof evidence (kernel
# trace + FETCH / WRITE / MFMA-busy PMC passes) for C3, C5 and C2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
head -c 300 gpurun_out/bench_default.json; echo
cp gpurun_out/bench_detail.json gpurun_out/bench_default_detail.json
for c in c3 c5 c2; do bash tools/gpu/profile.sh $c > gpurun_out/profile_$c.log 2>&1 || { tail -20 gpurun_out/profile_$c.log; exit 1; }; done
ls gpurun_out/prof_c3 gpurun_out/prof_c5 gpurun_out/prof_c2
