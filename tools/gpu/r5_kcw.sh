#!/bin/bash
# GPU box: DP tests with the in-launch weight-gradient combine, then per-rank C3
# (strong N=8 and weak N=8) with DDPG_KCOMB_WGRAD=1 / 0, interleaved
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dp.py tests/test_gpu_switches.py > gpurun_out/kcw_tests.log 2>&1 \
  || { tail -40 gpurun_out/kcw_tests.log; exit 1; }
tail -2 gpurun_out/kcw_tests.log
for r in 1 2; do for mode in strong weak; do for v in 1 0; do
  DDPG_KCOMB_WGRAD=$v timeout -k 10 300 python -u bench.py --config c3 --per-rank-of 8 --scaling $mode \
    --steps 30 --warmup 5 > gpurun_out/kcw_${mode}_${v}_$r.json 2> gpurun_out/kcw.err || { tail gpurun_out/kcw.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/kcw_${mode}_${v}_$r.json')); m=d['projected_scaling']['$mode']['8']
print('kc_wgrad=$v $mode r$r per-rank', m['step_ms'], m['gpu_busy_ms'], m['launches_per_step'], m['speedup_vs_1gpu'])"
done; done; done
