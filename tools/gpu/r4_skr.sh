#!/bin/bash
# GPU box: skinny kernel rows in flight: A = R 4 (default), B = R 6, C = R 8
set -o pipefail
mkdir -p gpurun_out
echo "== C3"; bash tools/gpu/ab.sh c3 2 2>&1 | tee gpurun_out/skr_ab_c3.txt || exit 1
for v in A B C; do python3 -c "
import json; d=json.load(open('gpurun_out/ab_c3_${v}_2.json')); print('$v', {k: v for k, v in d['kernels'].items() if k.startswith('skinny')})"; done
echo "== C5"; bash tools/gpu/ab.sh c5 2 2>&1 | tee gpurun_out/skr_ab_c5.txt || exit 1
for v in A B C; do python3 -c "
import json; d=json.load(open('gpurun_out/ab_c5_${v}_2.json')); print('$v', {k: v for k, v in d['kernels'].items() if k.startswith('skinny')})"; done
