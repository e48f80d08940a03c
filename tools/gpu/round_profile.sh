#!/bin/bash
# GPU box: the driver's default bench command, then rocprof evidence for C3 and C5
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
head -c 600 gpurun_out/bench_default.json; echo
bash tools/gpu/profile.sh c3 || exit $?
bash tools/gpu/profile.sh c5 || exit $?
