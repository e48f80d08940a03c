#!/bin/bash
# GPU box: the parity suite, then a same-box A/B of DDPG_GEMM256 values ($1, default "0 1 2") at C5
mkdir -p gpurun_out
[ -n "$NOTESTS" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/gputests.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "PASS|FAIL|ERROR" gpurun_out/gputests.log | tail -70
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 1 2; do
  for v in ${1:-0 1 2}; do
    DDPG_GEMM256=$v timeout -k 10 200 python -u bench.py --config c5 --no-cpu --no-small --steps 50 --warmup 10 > gpurun_out/g256_${v}_${r}.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/g256_${v}_${r}.json')); print('GEMM256=$v', $r, d['value'], d['step_latency']['median_ms'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['frac']); print({k: (v['avg_us'], v['per_step']) for k, v in d['kernels'].items() if k.startswith('gemm')})"
  done
done
