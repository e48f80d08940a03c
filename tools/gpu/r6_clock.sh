#!/bin/bash
# Clock reconciliation: one PMC pass per config with a wave-lifetime clock
# (SQ_WAVE_CYCLES quad-cycles / SQ_WAVES / duration), SQ_BUSY_CYCLES,
# SQ_CYCLES, GRBM_GUI_ACTIVE and SQ_VALU_MFMA_BUSY_CYCLES on the same dispatches
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/clk
rocprofv3 -L > gpurun_out/clk/counters.txt 2>&1 || true
for CFG in c3 c5; do
  ARGS="--config $CFG --no-cpu --no-small --no-project --steps 20 --warmup 5 --profile-steps 20"
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT \
    --kernel-trace --output-format csv -d gpurun_out/clk/$CFG -o run -- python3 bench.py $ARGS \
    > gpurun_out/clk/bench_$CFG.json 2> gpurun_out/clk/bench_$CFG.err || exit $?
done
ls -R gpurun_out/clk | head
