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
echo "== per-rank (rank 0 of 8) with DDPG_PAR=0 / 1"
for r in 1 2; do for p in 0 1; do
  DDPG_PAR=$p timeout -k 10 300 python -u bench.py --per-rank-of 8 --scaling strong --steps 30 --warmup 5 > gpurun_out/par${p}_pr8_$r.json 2> gpurun_out/par${p}_pr8_$r.err || { tail gpurun_out/par${p}_pr8_$r.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/par${p}_pr8_$r.json'))['projected_scaling']
print('PAR=$p', $r, 'strong8', d['strong']['8']['step_ms'], d['strong']['8']['speedup_vs_1gpu'], 'weak8', d['weak']['8']['step_ms'], d['weak']['8']['speedup_vs_1gpu'])"
done; done
