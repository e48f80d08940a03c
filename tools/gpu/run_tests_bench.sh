#!/bin/bash
# GPU box: parity suite, then (unless the suite crashed/hung) a short bench.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/gputests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -40 gpurun_out/gputests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
echo "bench rc=$brc"
cat gpurun_out/bench.json | head -c 3000
exit $brc
