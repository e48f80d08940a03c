#!/bin/bash
# GPU box: per-rank C3 strong N=8 with DDPG_GEMM_M16=0 / 1, interleaved
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for v in 1 0; do
  DDPG_GEMM_M16=$v timeout -k 10 300 python -u bench.py --config c3 --per-rank-of 8 --scaling strong --steps 30 --warmup 5 \
    > gpurun_out/r5_prab_$v_$r.json 2> gpurun_out/r5_prab.err || { tail gpurun_out/r5_prab.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r5_prab_$v_$r.json')); m=d['projected_scaling']['strong']['8']
print('m16=$v r$r per-rank', m['step_ms'], m['kernels_ms_per_step'])"
done; done
