#!/bin/bash
# GPU box: small downloads through pinned memory -- the 1:1 parity tests, then
# the 1:1 per-step latency A/B (A = words, B = DDPG_STATS_SPIN=0)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_switches.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_graph_pin.py -k "spin or train_methods or forward or mountaincar or graph" -x -q --timeout 200 --timeout-method thread > gpurun_out/rows.log 2>&1 || { tail -30 gpurun_out/rows.log; exit 1; }
tail -2 gpurun_out/rows.log
for i in 1 2; do
  timeout -k 10 120 python -u tools/gpu/oneone_lat.py 1000 | sed "s/^/A /" || exit 1
  DDPG_STATS_SPIN=0 timeout -k 10 120 python -u tools/gpu/oneone_lat.py 1000 | sed "s/^/B /" || exit 1
done
