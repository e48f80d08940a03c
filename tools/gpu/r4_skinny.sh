#!/bin/bash
# GPU box: full GPU suite, then same-box A/B of the skinny kernel's narrow
# rows through LDS (A = default, B = DDPG_SKINNY_NL=0, the scalar-load form)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sk_suite.log 2>&1
rc=$?; tail -2 gpurun_out/sk_suite.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/sk_suite.log | head -20; exit $rc; }
echo "== C3"; bash tools/gpu/envab.sh DDPG_SKINNY_NL=0 c3 3 skinny 2>&1 | tee gpurun_out/skinny_nl_ab_c3.txt || exit 1
echo "== C5"; bash tools/gpu/envab.sh DDPG_SKINNY_NL=0 c5 2 skinny 2>&1 | tee gpurun_out/skinny_nl_ab_c5.txt
