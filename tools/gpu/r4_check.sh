#!/bin/bash
# GPU box: the data-parallel / small-M tests first (new code paths), then the
# whole parity suite, then the default bench (unless a step failed).
# usage: tools/gpu/r4_check.sh [bench args...]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/dp_tests.log 2>&1
rc=$?
echo "dp tests rc=$rc"
tail -30 gpurun_out/dp_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/gputests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -15 gpurun_out/gputests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
echo "bench rc=$brc"
tail -5 gpurun_out/bench.err
python - <<'EOF'
import json
try:
    d = json.loads(open("gpurun_out/bench.json").read().strip().splitlines()[-1])
except Exception as e:
    print("no bench json", e); raise SystemExit(0)
print("value", d["value"], "ms", d["ms_per_step"], "roof", d["roofline"]["kernel"], d["roofline"]["frac"])
for k in ("small_batch", "c5_bf16"):
    if k in d: print(k, d[k]["value"], d[k]["ms_per_step"], d[k].get("step_latency"))
for blk in (d.get("projected_scaling"), d.get("c5_bf16", {}).get("projected_scaling")):
    if not blk: continue
    for mode in ("strong", "weak"):
        for n, m in blk[mode].items():
            print(mode, n, m["per_rank_batch"], m["step_ms"], m["window_us"], m["exposed_exchange_us"], m["speedup_vs_1gpu"])
EOF
exit $brc
