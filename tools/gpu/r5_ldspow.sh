#!/bin/bash
# GPU box: clock cost of LDS fragment reads under the power limit, and the
# 64x64 wave tile (tools/mfma_lds_power_bench.hip)
mkdir -p gpurun_out
timeout -k 10 120 ./tools/mfma_lds_power_bench > gpurun_out/ldspow.log 2>&1; rc=$?
cat gpurun_out/ldspow.log; exit $rc
