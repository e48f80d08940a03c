#!/bin/bash
# GPU box, round-6 final check: the whole GPU suite, smoke(), the driver's
# default bench command
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/final_tests.log 2>&1 || { tail -30 gpurun_out/final_tests.log; exit 1; }
tail -2 gpurun_out/final_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || exit $?
wc -c gpurun_out/final_bench.json
head -c 700 gpurun_out/final_bench.json
