#!/bin/bash
# GPU box: kernel-argument ring flushes -- their bitwise test and the replay /
# worker tests, then the worker-loop latency A/B (A = args, B = DDPG_RING_ARGS=0)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_switches.py tests/test_gpu_parity.py -k "ring_args or replay or worker or fused_learner or rejected or spin" -x -q --timeout 200 --timeout-method thread > gpurun_out/ring.log 2>&1 || { tail -30 gpurun_out/ring.log; exit 1; }
tail -2 gpurun_out/ring.log
for i in 1 2; do
  timeout -k 10 120 python -u tools/gpu/worker_lat.py 2000 2>/dev/null | sed "s/^/A /" || exit 1
  DDPG_RING_ARGS=0 timeout -k 10 120 python -u tools/gpu/worker_lat.py 2000 2>/dev/null | sed "s/^/B /" || exit 1
done
