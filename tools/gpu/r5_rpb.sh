#!/bin/bash
# GPU box: thin_k row tiles per block (DDPG_TK_RPB = auto / 2 / 4), C3, interleaved;
# per-call-site thin_k times from the bench's profile pass
mkdir -p gpurun_out
for r in 1 2; do for v in 0 2 4; do
  if [ $v = 0 ]; then unset DDPG_TK_RPB; else export DDPG_TK_RPB=$v; fi
  timeout -k 10 200 python -u bench.py --config c3 --no-cpu --no-small --no-project --steps 50 \
    --warmup 10 > gpurun_out/rpb_${v}_$r.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/rpb_${v}_$r.json'))
print('rpb=$v r$r', d['value'], d['gpu_busy_ms_per_step'], {k:v['avg_us'] for k,v in d['kernels_by_phase'].items() if k.startswith('thin_k')})"
done; done
