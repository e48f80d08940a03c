#!/bin/bash
# GPU box: the final build: full GPU suite, smoke(), default bench, C3 profile passes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/last_suite.log 2>&1
rc=$?; tail -2 gpurun_out/last_suite.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/last_suite.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/last_smoke.log 2>&1 || { tail gpurun_out/last_smoke.log; exit 1; }
tail -1 gpurun_out/last_smoke.log
T0=$(date +%s); timeout -k 10 400 python -u bench.py > gpurun_out/bench_last.json 2> gpurun_out/bench_last.err || { tail gpurun_out/bench_last.err; exit 1; }; echo "bench wall $(( $(date +%s) - T0 )) s"
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/bench_last.json"))
print("C3", d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["avg_launch_us"], d["roofline"]["frac"], d["roofline"]["traffic"])
c5 = d.get("c5_bf16", {})
print("C5", c5.get("value"), c5.get("ms_per_step"), c5.get("roofline", {}).get("kernel"), c5.get("roofline", {}).get("frac"), c5.get("roofline", {}).get("traffic"))
sb = d.get("small_batch", {})
print("C2", sb.get("value"), sb.get("step_latency"))
print("strong8", d["projected_scaling"]["strong"]["8"]["speedup_vs_1gpu"], "weak8", d["projected_scaling"]["weak"]["8"]["speedup_vs_1gpu"])
PY
bash tools/gpu/profile.sh c3 > gpurun_out/profile_c3_last.log 2>&1 || { tail -20 gpurun_out/profile_c3_last.log; exit 1; }
head -12 gpurun_out/prof_c3/kernels_c3.txt
