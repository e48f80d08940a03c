#!/bin/bash
# GEMM microbench + PMC passes on one case (tuning aid)
export TMPDIR=/tmp
O=gpurun_out/gpmc; rm -rf $O; mkdir -p $O
timeout -k 10 120 ./tools/gemm_bench > $O/bench.txt 2>&1 || exit $?
cat $O/bench.txt
CASE=${1:-"fwd K=1024"}
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum" \
         "SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/p$i -o run -- ./tools/gemm_bench "$CASE" > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/gpmc/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print("   %-28s %14.4g  (n=%d)" % (c, sum(v) / len(v), len(v)))
PY
