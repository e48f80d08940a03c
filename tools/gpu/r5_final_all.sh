#!/bin/bash
# GPU box: smoke(), the driver's default bench, rocprof evidence for C3 / C5 / C2, per-rank C3 strong
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash tools/gpu/r5_final_prof.sh
