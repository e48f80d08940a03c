#!/bin/bash
# GPU box: DP tests, then per-rank projections (C3 weak/strong N=8, C5 weak N=2/8)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_switches.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r5_dp.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/r5_dp.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r5_dp.log | head -20; tail -40 gpurun_out/r5_dp.log; exit $rc; }
for spec in "c3 weak 8" "c3 strong 8" "c5 weak 8" "c5 weak 2"; do
  set -- $spec
  timeout -k 10 300 python -u bench.py --config $1 --per-rank-of $3 --scaling $2 --steps 30 --warmup 5 \
    > gpurun_out/r5_pr_$1_$2_$3.json 2> gpurun_out/r5_pr_$1_$2_$3.err || { tail gpurun_out/r5_pr_$1_$2_$3.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r5_pr_$1_$2_$3.json')); m=d['projected_scaling']['$2']['$3']
print('$spec', 'base', d['projected_scaling']['measured_1gpu_updates_s'], 'per-rank', m['step_ms'], m['step_mode'], m['window_us'], 'exposed', m['exposed_exchange_us'], 'x', m['speedup_vs_1gpu'], 'pess', m['pessimistic_speedup'])"
done
