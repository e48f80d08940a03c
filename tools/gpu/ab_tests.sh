#!/bin/bash
# GPU box: parity suite against every tools/ab/lib<X>.so, then the same-box A/B bench
# (bash tools/gpu/ab_tests.sh [config] [rounds])
mkdir -p gpurun_out
for L in tools/ab/lib*.so; do
  v=$(basename $L .so)
  DDPG_LIB_PATH=$L timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/abtests_$v.log 2>&1 || { tail -30 gpurun_out/abtests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/abtests_$v.log)"
done
bash tools/gpu/ab.sh ${1:-c3} ${2:-3}
