#!/bin/bash
# gemm_h microbench + PMC passes on the cases matching $1 (tuning aid)
export TMPDIR=/tmp
O=gpurun_out/hpmc; rm -rf $O; mkdir -p $O
CASE=${1:-"c5 fwd"}
timeout -k 10 120 ./tools/gemmh_bench "$CASE" > $O/bench.txt 2>&1 || exit $?
cat $O/bench.txt
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/p$i -o run -- ./tools/gemmh_bench "$CASE" > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/hpmc/p*/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gemm_h" not in r["Kernel_Name"]: continue
        agg[r["Kernel_Name"][:70] + " grid=" + r.get("Grid_Size", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print("   %-28s %14.4g  (n=%d)" % (c, sum(v) / len(v), len(v)))
PY
