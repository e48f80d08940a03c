#!/bin/bash
# GPU box: thin_k column-block variants (isolated), the full GPU suite,
# shape-keyed C5 / C3 step profiles, then the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/thin_k_bench > gpurun_out/tk_c128.txt 2>&1 && timeout -k 10 120 ./tools/thin_k_bench_c64 > gpurun_out/tk_c64.txt 2>&1 || { tail gpurun_out/tk_c64.txt; exit 1; }
for f in tk_c128 tk_c64; do echo "== $f"; grep -A40 "8 row tiles" gpurun_out/$f.txt | grep -A1 "5 parts twin-only"; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r4_suite.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r4_suite.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r4_suite.log | head -20; tail -30 gpurun_out/r4_suite.log; exit $rc; }
timeout -k 10 200 python -u tools/gpu/keys.py c5 20 > gpurun_out/keys_c5_pack.txt 2> gpurun_out/keys_c5_pack.err || { tail gpurun_out/keys_c5_pack.err; exit 1; }
head -14 gpurun_out/keys_c5_pack.txt; tail -1 gpurun_out/keys_c5_pack.txt
timeout -k 10 200 python -u tools/gpu/keys.py c3 20 > gpurun_out/keys_c3_r4.txt 2> gpurun_out/keys_c3_r4.err || { tail gpurun_out/keys_c3_r4.err; exit 1; }
grep thin_k gpurun_out/keys_c3_r4.txt; tail -1 gpurun_out/keys_c3_r4.txt
T0=$(date +%s); timeout -k 10 400 python -u bench.py > gpurun_out/bench_r4.json 2> gpurun_out/bench_r4.err || { tail gpurun_out/bench_r4.err; exit 1; }; echo "bench wall $(( $(date +%s) - T0 )) s"
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/bench_r4.json"))
print("C3", d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["avg_launch_us"], d["roofline"]["frac"])
c5 = d.get("c5_bf16", {})
print("C5", c5.get("value"), c5.get("ms_per_step"), c5.get("roofline", {}).get("kernel"), c5.get("roofline", {}).get("frac"))
sb = d.get("small_batch", {})
print("C2", sb.get("value"), sb.get("step_latency"))
print("strong8", d["projected_scaling"]["strong"]["8"]["speedup_vs_1gpu"], "weak8", d["projected_scaling"]["weak"]["8"]["speedup_vs_1gpu"])
PY
echo "== A/B: A = round-4 commit a3be9e4, B = + one-pass epilogue + slab_sum loads ahead"; bash tools/gpu/ab.sh c3 3 2>&1 | tee gpurun_out/epi1pass_ab_c3.txt
