#!/bin/bash
# GPU box: parity suite, then C3 and C5 bench lines (no CPU leg)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/gputests.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/gputests.log | tail -45
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit $?
timeout -k 10 200 python -u bench.py --config c5 --steps 30 --warmup 5 --no-cpu --no-small > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || exit $?
python3 - <<'PY'
import json
for c in ("c3", "c5"):
    d = json.load(open("gpurun_out/bench_%s.json" % c))
    print(c, d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["avg_launch_us"], d["roofline"]["frac"])
    for k, v in list(d["kernels_by_phase"].items())[:14]:
        print("   ", k, v)
    if "small_batch" in d: print("  small", d["small_batch"]["ms_per_step"])
PY
