#!/bin/bash
# GPU box: small-M combine with up to 8 splits: DP tests at cap 8, then the
# per-rank strong step (rank 0 of 8 and of 4) at caps 4 and 8, and the kc microbench
set -o pipefail
mkdir -p gpurun_out
DDPG_KCOMB_SPLITS=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s8_tests.log 2>&1
rc=$?; tail -1 gpurun_out/s8_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/s8_tests.log | head; exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_switches.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s4_tests.log 2>&1 || { tail gpurun_out/s4_tests.log; exit 1; }
tail -1 gpurun_out/s4_tests.log
for r in 1 2; do for sp in 4 8; do
  DDPG_KCOMB_SPLITS=$sp timeout -k 10 300 python -u bench.py --per-rank-of 8 --scaling strong --steps 30 --warmup 5 > gpurun_out/s${sp}_pr8_$r.json 2> gpurun_out/s${sp}_pr8_$r.err || { tail gpurun_out/s${sp}_pr8_$r.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/s${sp}_pr8_$r.json'))['projected_scaling']
m=d['strong']['8']; print('S<=$sp', $r, 'per-rank', m['step_ms'], 'speedup', m['speedup_vs_1gpu']); print('  ', {k: v for k, v in m['kernels_ms_per_step'].items() if k.startswith('gemm')})"
done; done
