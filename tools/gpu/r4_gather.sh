#!/bin/bash
# GPU box: GPU suite subset, then A/B of the gather's coalesced slot reads (A = per-wave reads, B = per block)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g_suite.log 2>&1
rc=$?; tail -1 gpurun_out/g_suite.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/g_suite.log | head -20; exit $rc; }
echo "== C3"; bash tools/gpu/ab.sh c3 2 2>&1 | tee gpurun_out/gather_ab_c3.txt || exit 1
for v in A B; do python3 -c "
import json; d=json.load(open('gpurun_out/ab_c3_${v}_2.json')); print('$v', {k: v for k, v in d['kernels'].items() if k.startswith(('gather','critic_head','actor_out'))})"; done
echo "== C5"; bash tools/gpu/ab.sh c5 2 2>&1 | tee gpurun_out/gather_ab_c5.txt || exit 1
for v in A B; do python3 -c "
import json; d=json.load(open('gpurun_out/ab_c5_${v}_2.json')); print('$v', {k: v for k, v in d['kernels'].items() if k.startswith(('gather','critic_head','actor_out'))})"; done
