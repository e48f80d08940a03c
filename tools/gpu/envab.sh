#!/bin/bash
# same-box A/B of an environment switch: A = default, B = $1
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in A B; do
    if [ $v = B ]; then export $1; else unset ${1%%=*}; fi
    timeout -k 10 200 python -u bench.py --config ${2:-c3} --no-cpu --no-small --steps 50 --warmup 10 > gpurun_out/eab_${v}_${r}.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/eab_${v}_${r}.json')); print('$v', $r, d['value'], d['step_latency']['median_ms'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
  done
done
