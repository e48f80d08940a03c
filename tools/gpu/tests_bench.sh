#!/bin/bash
# GPU box: parity suite, then the driver's default bench command.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -3 gpurun_out/gputests.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/bench_default.json'))
print('C3', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline']['traffic'])
print('C5', d['c5_bf16']['value'], d['c5_bf16']['ms_per_step'], d['c5_bf16']['roofline']['frac'])
print('C2', d['small_batch']['value'], d['small_batch']['ms_per_step'])"
