#!/bin/bash
# GPU box: same-box comparison of builds of the library (tools/ab/lib<X>.so,
# X = A, B, C, ...), interleaved bench runs: bash tools/gpu/ab.sh [config] [rounds]
CFG=${1:-c3}; R=${2:-3}
mkdir -p gpurun_out
AB=${AB_DIR:-tools/ab}
VS=$(cd $AB && ls lib*.so | sed 's/^lib//; s/\.so$//')
for r in $(seq 1 $R); do
  for v in $VS; do
    DDPG_LIB_PATH=$AB/lib$v.so timeout -k 10 200 python -u bench.py --config $CFG --no-cpu --no-small --no-project \
      --steps 50 --warmup 10 > gpurun_out/ab_${CFG}_${v}_$r.json 2> gpurun_out/ab_${CFG}_${v}_$r.err || exit $?
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_${CFG}_${v}_$r.json')); print('$v', $r, d['value'], d['ms_per_step'], d['step_latency']['median_ms'], d['kernels'].get('adam+reduce+soft_update'))"
  done
done
