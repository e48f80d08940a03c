#!/bin/bash
# same-box A/B of an environment switch: A = default, B = $1 (VAR=value)
# usage: tools/gpu/envab.sh VAR=value [config] [rounds] [kernel-prefix to report]
mkdir -p gpurun_out
CFG=${2:-c3}
ROUNDS=${3:-3}
KPFX=${4:-}
for r in $(seq 1 $ROUNDS); do
  for v in A B; do
    if [ $v = B ]; then export $1; else unset ${1%%=*}; fi
    timeout -k 10 200 python -u bench.py --config $CFG --no-cpu --no-small --no-project --steps 50 \
      --warmup 10 > gpurun_out/eab_${CFG}_${v}_${r}.json 2>/dev/null || exit $?
    python3 - "$v" "$r" "$CFG" "$KPFX" <<'EOF'
import json, sys
v, r, cfg, kp = sys.argv[1:5]
d = json.load(open("gpurun_out/eab_%s_%s_%s.json" % (cfg, v, r)))
ks = ""
if kp:
    # compact contract line: kernels as {name: [avg_us, per_step]}
    ks = " ".join("%s=%.2fus*%g" % (k.split("<")[0], x[0], x[1])
                  for k, x in d["kernels"].items() if k.startswith(kp))
print(v, r, d["value"], d["step_latency"]["median_ms"], d["roofline"]["kernel"],
      d["roofline"]["avg_launch_us"], d["roofline"]["frac"], ks, flush=True)
EOF
  done
done
