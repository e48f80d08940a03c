#!/bin/bash
# GPU box: small-M combine (sc1 hand-off) + thin_k register epilogue:
# tests, per-rank projection at N=8 strong, then thin_k A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_switches.py tests/test_gpu_graph_pin.py \
  tests/test_gpu_configs.py -x -v --timeout 120 --timeout-method thread > gpurun_out/kc_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/kc_tests.log | tail -8
[ $rc -eq 0 ] || { tail -40 gpurun_out/kc_tests.log; exit $rc; }
timeout -k 10 300 python -u bench.py --per-rank-of 8 --scaling strong --steps 30 --warmup 5 \
  > gpurun_out/pr8.json 2> gpurun_out/pr8.err || { tail gpurun_out/pr8.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/pr8.json')); m=d['projected_scaling']['strong']['8']
print('base', d['projected_scaling']['measured_1gpu_updates_s'], 'per-rank', m['step_ms'], m['gpu_busy_ms'], m['window_us'], m['speedup_vs_1gpu']); print(m['kernels_ms_per_step'])"
bash tools/gpu/envab.sh DDPG_TK_LDS=1 c3 2 thin_k 2>&1 | tee gpurun_out/tk_ab_c3.txt || exit $?
bash tools/gpu/envab.sh DDPG_TK_LDS=1 c5 1 thin_k 2>&1 | tee gpurun_out/tk_ab_c5.txt
