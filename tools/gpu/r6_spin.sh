#!/bin/bash
# GPU box: the completion-word reads -- their bitwise tests, then the C2
# synchronous latency A/B (A = words, B = DDPG_STATS_SPIN=0)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_switches.py tests/test_gpu_parity.py -k "spin or fused_learner or action_selection or small_batch_path or graph_replay" -x -q --timeout 200 --timeout-method thread > gpurun_out/spin.log 2>&1 || { tail -30 gpurun_out/spin.log; exit 1; }
tail -2 gpurun_out/spin.log
for r in 1 2; do
  timeout -k 10 120 python -u tools/gpu/c2_sync_lat.py c2 2000 2>/dev/null | sed "s/^/A /" || exit 1
  DDPG_STATS_SPIN=0 timeout -k 10 120 python -u tools/gpu/c2_sync_lat.py c2 2000 2>/dev/null | sed "s/^/B /" || exit 1
done
