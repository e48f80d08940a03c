#!/bin/bash
# GPU box: per-phase stamps of the full-size C3 forward twin GEMM, then a
# short C3-only bench of the current library (same box reference).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/h3_phase_bench > gpurun_out/h3_phase.txt 2>&1 || { cat gpurun_out/h3_phase.txt; exit 1; }
cat gpurun_out/h3_phase.txt
exit 0
timeout -k 10 200 python -u bench.py --config c3 --no-cpu --no-small --no-project --steps 50 --warmup 10 \
  > gpurun_out/r5_c3_base.json 2> gpurun_out/r5_c3_base.err || { tail gpurun_out/r5_c3_base.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5_c3_base.json')); print(d['value'], d['ms_per_step'], d['roofline'])"
