#!/bin/bash
# GPU box: LDS bank-conflict counters per kernel at C5 and C3 (one PMC pass each)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in c5 c3; do
  rm -rf gpurun_out/pmc_lds_$cfg
  timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace \
    --output-format csv -d gpurun_out/pmc_lds_$cfg -o run -- python3 bench.py --config $cfg --no-cpu \
    --no-small --no-project --steps 10 --warmup 3 --profile-steps 5 > gpurun_out/pmc_lds_$cfg.json \
    2> gpurun_out/pmc_lds_$cfg.err || { tail gpurun_out/pmc_lds_$cfg.err; exit 1; }
  F=$(find gpurun_out/pmc_lds_$cfg -name 'run_counter_collection.csv' | head -1)
  python3 - "$F" <<'PY'
import collections, csv, sys
sys.path.insert(0, "profiles")
from pmc_traffic import bench_name
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
seen = set()
for r in csv.DictReader(open(sys.argv[1])):
    k = bench_name(r["Kernel_Name"])
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    d = (k, r.get("Dispatch_Id") or r.get("Correlation_Id"))
    if d not in seen:
        seen.add(d); n[k] += 1
for k in sorted(agg, key=lambda k: -agg[k].get("SQ_LDS_IDX_ACTIVE", 0)):
    a = agg[k]; act = a.get("SQ_LDS_IDX_ACTIVE", 0)
    if act <= 0: continue
    print("%-45s launches %4d  conflict/active %.3f  active cycles/launch %.0f" % (
        k[:45], n[k], a.get("SQ_LDS_BANK_CONFLICT", 0) / act, act / n[k]))
PY
done
