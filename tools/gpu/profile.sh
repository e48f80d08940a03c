#!/bin/bash
# GPU box: rocprofv3 evidence for one bench configuration (default c3):
#   1. kernel trace + --stats of the bench command
#   2. PMC FETCH_SIZE pass, 3. PMC WRITE_SIZE pass, 4. PMC MFMA-busy pass (separate
#      runs, gfx950 counter limits)
#   5. profiles/pmc_mfma.py + pmc_traffic.py + summarize.py -> gpurun_out/prof_<cfg>/
# usage: bash tools/gpu/profile.sh [config] [extra bench args...]
set -o pipefail
CFG=${1:-c3}; shift
export TMPDIR=/tmp
OUT=gpurun_out/prof_$CFG
rm -rf $OUT; mkdir -p $OUT
ARGS="--config $CFG --no-cpu --no-small --no-project --steps 20 --warmup 5 --profile-steps 20 $*"
# fused steps per run: warmup + steps + latency pass (20) + profile pass (20)
NSTEPS=65
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py $ARGS \
  > $OUT/bench_trace.json 2> $OUT/bench_trace.err || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o run \
  -- python3 bench.py $ARGS > $OUT/bench_fetch.json 2> $OUT/bench_fetch.err || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o run \
  -- python3 bench.py $ARGS > $OUT/bench_write.json 2> $OUT/bench_write.err || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace \
  --output-format csv -d $OUT/pmc_mfma -o run -- python3 bench.py $ARGS > $OUT/bench_mfma.json \
  2> $OUT/bench_mfma.err || exit $?
M=$(dirname $(find $OUT/pmc_mfma -name 'run_counter_collection.csv' | head -1))
python3 profiles/pmc_mfma.py $M $CFG $NSTEPS > $OUT/mfma_$CFG.json || exit $?
F=$(dirname $(find $OUT/pmc_fetch -name 'run_counter_collection.csv' | head -1))
W=$(dirname $(find $OUT/pmc_write -name 'run_counter_collection.csv' | head -1))
python3 profiles/pmc_traffic.py $F $W $CFG $NSTEPS > $OUT/pmc_$CFG.json || exit $?
DB=$(find $OUT/trace -name '*results.db' | head -1)
if [ -n "$DB" ]; then python3 profiles/summarize.py $DB > $OUT/kernels_$CFG.txt; fi
find $OUT/trace -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_$CFG.csv \;
ls -R $OUT | head -40
cat $OUT/bench_trace.json | head -c 1500
