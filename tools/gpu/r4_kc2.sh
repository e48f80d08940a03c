#!/bin/bash
# GPU box: small-M combine with all partials in flight: microbench, tests,
# then the per-rank (N=8 strong) step at split caps 2 / 3 / 4.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/kc_bench > gpurun_out/kc_bench2.txt 2>&1 || { cat gpurun_out/kc_bench2.txt; exit 1; }
cat gpurun_out/kc_bench2.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_switches.py tests/test_gpu_graph_pin.py \
  tests/test_gpu_configs.py -x -v --timeout 120 --timeout-method thread > gpurun_out/kc2_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/kc2_tests.log | tail -3
[ $rc -eq 0 ] || { tail -40 gpurun_out/kc2_tests.log; exit $rc; }
for s in 2 3 4; do
  DDPG_KCOMB_SPLITS=$s timeout -k 10 300 python -u bench.py --per-rank-of 8 --scaling strong --steps 30 --warmup 5 \
    > gpurun_out/pr8_s$s.json 2> gpurun_out/pr8_s$s.err || { tail gpurun_out/pr8_s$s.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/pr8_s$s.json')); m=d['projected_scaling']['strong']['8']
print('S<=$s base', d['projected_scaling']['measured_1gpu_updates_s'], 'per-rank', m['step_ms'], m['gpu_busy_ms'], m['window_us'], m['speedup_vs_1gpu']); print(m['kernels_ms_per_step'])"
done
