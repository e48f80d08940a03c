#!/bin/bash
# GPU box: the GPU suite on the 64-column thin_k build, then same-box A/B
# (B = default 128-column thin_k, C = 64-column) at C3 and C5
set -o pipefail
mkdir -p gpurun_out
DDPG_LIB_PATH=tools/ab/libC.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c64_suite.log 2>&1
rc=$?; tail -2 gpurun_out/c64_suite.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/c64_suite.log | head -20; exit $rc; }
echo "== C3"; bash tools/gpu/ab.sh c3 2 2>&1 | tee gpurun_out/c64_ab_c3.txt || exit 1
echo "== C5"; bash tools/gpu/ab.sh c5 2 2>&1 | tee gpurun_out/c64_ab_c5.txt || exit 1
for v in B C; do python3 -c "
import json; d=json.load(open('gpurun_out/ab_c3_${v}_2.json')); print('$v', {k: v for k, v in d['kernels'].items() if k.startswith('thin_k')})"; done
echo "==== closing evidence"; bash tools/gpu/r4_final.sh
