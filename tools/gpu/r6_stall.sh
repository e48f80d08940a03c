#!/bin/bash
# Stall composition of the step's kernels: one SQ PMC pass per config
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/stall
for CFG in c3 c5; do
  ARGS="--config $CFG --no-cpu --no-small --no-project --steps 20 --warmup 5 --profile-steps 20"
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES \
    --kernel-trace --output-format csv -d gpurun_out/stall/$CFG -o run -- python3 bench.py $ARGS \
    > gpurun_out/stall/bench_$CFG.json 2> gpurun_out/stall/bench_$CFG.err || exit $?
done
