"""Stall composition per kernel from one SQ PMC pass (tools/gpu/r6_stall.sh):

  python profiles/pmc_stall.py <pmc_dir>

SQ_WAIT_ANY (wave parked: s_waitcnt / barrier), SQ_WAIT_INST_ANY (issue stall),
SQ_ACTIVE_INST_ANY (issuing) as fractions of SQ_WAVE_CYCLES (they are disjoint
and sum to about it, MI355X_MICROARCH.md PMC table); SQ_WAIT_INST_LDS (an
issue-stall sub-bucket); LDS bank-conflict cycles over LDS-array cycles.
"""
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import bench_name  # noqa: E402


def main(d):
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    dur = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        k = (bench_name(r["Kernel_Name"]), r["Grid_Size"], r["Dispatch_Id"])
        per[k[:2]][k[2]][r["Counter_Name"]] = float(r["Counter_Value"])
        dur[k] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    print("# %s" % d)
    print("# kernel | grid | avg us | wait_any | wait_inst_any | active_inst | "
          "wait_inst_lds | lds conflict / lds active")
    rows = []
    for (name, grid), disp in per.items():
        n = len(disp)
        s = lambda c: sum(x.get(c, 0.0) for x in disp.values())
        D = sum(dur[(name, grid, i)] for i in disp) / n / 1e3
        wc = s("SQ_WAVE_CYCLES")
        if D < 5 or not wc:
            continue
        rows.append((D * n, "%s | %s | %.2f | %.3f | %.3f | %.3f | %.3f | %.3f" % (
            name, grid, D, s("SQ_WAIT_ANY") / wc, s("SQ_WAIT_INST_ANY") / wc,
            s("SQ_ACTIVE_INST_ANY") / wc, s("SQ_WAIT_INST_LDS") / wc,
            s("SQ_LDS_BANK_CONFLICT") / max(s("SQ_LDS_IDX_ACTIVE"), 1))))
    for _, line in sorted(rows, reverse=True):
        print(line)


if __name__ == "__main__":
    main(sys.argv[1])
