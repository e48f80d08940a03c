#!/bin/bash
# GPU box: the GPU test suite, then the default bench (contract line on stdout,
# full record in gpurun_out/bench_detail.json)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/r6_tests.log 2>&1 || { tail -30 gpurun_out/r6_tests.log; exit 1; }
tail -3 gpurun_out/r6_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/r6_bench.json 2> gpurun_out/r6_bench.err || exit $?
wc -c gpurun_out/r6_bench.json
head -c 3000 gpurun_out/r6_bench.json
