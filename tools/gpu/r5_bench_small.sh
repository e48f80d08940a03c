#!/bin/bash
# GPU box: GPU suite (hygiene changes), then the default bench (C3 + C5 + small batch + projections)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r5_gputests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/r5_gputests.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r5_gputests.log | head -20; tail -30 gpurun_out/r5_gputests.log; exit $rc; }
timeout -k 10 400 python -u bench.py > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err || { tail -20 gpurun_out/r5_bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r5_bench.json"))
print("C3", d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["avg_launch_us"], d["roofline"]["frac"])
print("C5", d["c5_bf16"]["value"], d["c5_bf16"]["ms_per_step"])
sb = d["small_batch"]
print("C2 B=64", sb["value"], sb["ms_per_step"], sb["step_latency"])
print("C2 B=256", json.dumps(sb["b256"])[:1500])
PY
