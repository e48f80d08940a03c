"""Clock reconciliation from one rocprofv3 PMC pass (tools/gpu/r6_clock.sh):

  python profiles/pmc_clock.py <pmc_dir> > profiles/r6/clock_<config>.txt

Per kernel (dispatch averages over the pass), beside the dispatch duration D
from the same records:
  wave clock   = 4 x SQ_WAVE_CYCLES / SQ_WAVES / D   (SQ_WAVE_CYCLES counts
                 quad-cycles per wave, MI355X_MICROARCH.md cycle-constants
                 table; a wave lives at most D, so this is a LOWER bound of the
                 shader clock, tight for one-round grids whose waves span the
                 dispatch)
  grbm clock   = GRBM_GUI_ACTIVE / 8 / D            (reads high on dispatches
                 shorter than ~0.3 ms, MI355X_MICROARCH.md 'DVFS give-back')
  count clock  = GRBM_COUNT / 8 / D                 (the same window, free-running)
  SQ_BUSY_CYCLES / D and SQ_CYCLES / D as reported
  mfma busy    = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x D x clock) at the
                 wave clock and at the 2.4 GHz peak
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
    rows = []
    for (name, grid), disp in per.items():
        n = len(disp)
        avg = lambda c: sum(x.get(c, 0.0) for x in disp.values()) / n
        D = sum(dur[(name, grid, i)] for i in disp) / n  # ns
        if D < 5000:
            continue
        wc = 4 * avg("SQ_WAVE_CYCLES") / max(avg("SQ_WAVES"), 1) / D
        mb = avg("SQ_VALU_MFMA_BUSY_CYCLES")
        rows.append((D * n, name, grid, n, D / 1e3, wc, avg("GRBM_GUI_ACTIVE") / 8 / D,
                     avg("GRBM_COUNT") / 8 / D, avg("SQ_BUSY_CYCLES") / D, avg("SQ_CYCLES") / D,
                     mb / (1024 * D * wc) if wc else 0.0, mb / (1024 * D * 2.4)))
    print("# %s" % d)
    print("# kernel | grid | dispatches | avg us | wave clock GHz (lower bound) | grbm GHz | "
          "count GHz | SQ_BUSY_CYCLES/ns | SQ_CYCLES/ns | mfma busy @wave clock | @2.4 GHz")
    for r in sorted(rows, reverse=True):
        print("%s | %s | %d | %.2f | %.3f | %.3f | %.3f | %.3f | %.3f | %.3f | %.3f" % r[1:])


if __name__ == "__main__":
    main(sys.argv[1])
