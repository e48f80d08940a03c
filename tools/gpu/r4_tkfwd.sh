#!/bin/bash
# GPU box: thin_k forward form + fast elu: microbench, full GPU suite, C3/C5 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/thin_k_bench > gpurun_out/tk_fwd.txt 2>&1 || { tail gpurun_out/tk_fwd.txt; exit 1; }
grep -A14 "6 row tiles" gpurun_out/tk_fwd.txt | grep -A2 "5 parts"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
rc=$?
echo "gpu suite rc=$rc"; grep -E "passed|failed" gpurun_out/gpu_suite.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gpu_suite.log | head; tail -30 gpurun_out/gpu_suite.log; exit $rc; }
timeout -k 10 400 python -u bench.py --steps 50 --warmup 10 > gpurun_out/bench_tkfwd.json 2> gpurun_out/bench_tkfwd.err || { tail gpurun_out/bench_tkfwd.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/bench_tkfwd.json"))
print("C3", d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["avg_launch_us"], d["roofline"]["frac"])
for k, v in d["kernels"].items():
    if k.startswith("thin_k"): print("  ", k, v)
c5 = d.get("c5_bf16", {})
print("C5", c5.get("value"), c5.get("ms_per_step"), c5.get("roofline", {}).get("frac"))
for k, v in c5.get("kernels", {}).items():
    if k.startswith("thin_k"): print("  ", k, v)
sb = d.get("small_batch", {})
print("C2", sb.get("value"), sb.get("step_latency"))
print("proj", json.dumps(d.get("projected_scaling", {}))[:600])
PY
