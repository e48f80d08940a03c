#!/bin/bash
# GPU box: DP tests (small path under a communicator), then the per-rank C2 B=256 step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_switches.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r5_dp.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/r5_dp.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r5_dp.log | head -20; tail -40 gpurun_out/r5_dp.log; exit $rc; }
timeout -k 10 300 python -u bench.py --config c2b --per-rank-of 8 --scaling weak --steps 200 --warmup 20 \
  > gpurun_out/r5_pr8_c2b.json 2> gpurun_out/r5_pr8_c2b.err || { tail gpurun_out/r5_pr8_c2b.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r5_pr8_c2b.json')); m=d['projected_scaling']['weak']['8']
print('base', d['projected_scaling']['measured_1gpu_updates_s'], 'per-rank', m['step_ms'], m['path'], m['step_mode'], m['window_us'], m['exposed_exchange_us'], m['speedup_vs_1gpu']); print(m['kernels_ms_per_step'])"
