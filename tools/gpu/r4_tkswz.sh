#!/bin/bash
# GPU box: GPU suite, LDS conflicts of thin_k with the new output-tile swizzle, A/B (A = old, B = new)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tks_suite.log 2>&1
rc=$?; tail -1 gpurun_out/tks_suite.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/tks_suite.log | head -20; exit $rc; }
bash tools/gpu/r4_lds.sh 2>&1 | grep -E "thin_k" || exit 1
echo "== C3"; bash tools/gpu/ab.sh c3 2 2>&1 | tee gpurun_out/tkswz_ab_c3.txt || exit 1
for v in A B; do python3 -c "
import json; d=json.load(open('gpurun_out/ab_c3_${v}_2.json')); print('$v', {k: v for k, v in d['kernels'].items() if k.startswith('thin_k')})"; done
echo "== C5"; bash tools/gpu/ab.sh c5 2 2>&1 | tee gpurun_out/tkswz_ab_c5.txt || exit 1
