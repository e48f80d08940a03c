#!/bin/bash
# GPU box: rocprofv3 passes for C5 and C2, the default bench line, then the
# slot-upload A/B at C3 / C5
set -o pipefail
mkdir -p gpurun_out
for cfg in c5 c2; do
  bash tools/gpu/profile.sh $cfg > gpurun_out/profile_$cfg.log 2>&1 || { tail -20 gpurun_out/profile_$cfg.log; exit 1; }
  echo "== $cfg"; head -8 gpurun_out/prof_$cfg/kernels_$cfg.txt
done
T0=$(date +%s); timeout -k 10 400 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail gpurun_out/bench_final.err; exit 1; }; echo "bench wall $(( $(date +%s) - T0 )) s"
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/bench_final.json"))
print("C3", d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["avg_launch_us"], d["roofline"]["frac"], d["roofline"]["traffic"], d.get("mfma_busy_step_counter"))
c5 = d.get("c5_bf16", {})
print("C5", c5.get("value"), c5.get("ms_per_step"), c5.get("roofline", {}).get("kernel"), c5.get("roofline", {}).get("frac"), c5.get("roofline", {}).get("traffic"))
sb = d.get("small_batch", {})
print("C2", sb.get("value"), sb.get("step_latency"))
print("strong8", d["projected_scaling"]["strong"]["8"]["speedup_vs_1gpu"], "weak8", d["projected_scaling"]["weak"]["8"]["speedup_vs_1gpu"])
PY
echo "== DDPG_SLOTS_H2D=1 A/B (slots uploaded vs read in place from pinned host memory)"
bash tools/gpu/envab.sh DDPG_SLOTS_H2D=1 c3 2 gather 2>&1 | tee gpurun_out/slots_ab_c3.txt
bash tools/gpu/envab.sh DDPG_SLOTS_H2D=1 c5 2 gather 2>&1 | tee gpurun_out/slots_ab_c5.txt
