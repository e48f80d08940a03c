#!/bin/bash
# GPU box: round-4 rocprofv3 evidence (kernel trace + stats, FETCH / WRITE /
# MFMA-busy PMC passes) for C3, C5 and C2 via tools/gpu/profile.sh
set -o pipefail
for cfg in c3 c5 c2; do
  bash tools/gpu/profile.sh $cfg > gpurun_out/profile_$cfg.log 2>&1 || { tail -20 gpurun_out/profile_$cfg.log; exit 1; }
  echo "== $cfg"; head -8 gpurun_out/prof_$cfg/kernels_$cfg.txt
done
