"""Per-kernel MFMA busy fraction from one rocprofv3 PMC pass.

  python profiles/pmc_mfma.py <pmc_dir> <config> <steps> > profiles/rN_mfma_<config>.json

The pass collects SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE (plus
SQ_BUSY_CYCLES) for every dispatch of the bench command, e.g.

  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES \
      --kernel-trace --output-format csv -d gpurun_out/pmc_mfma -o run -- python3 bench.py ...

Units (MI355X_MICROARCH.md, PMC table): SQ_VALU_MFMA_BUSY_CYCLES is a device
sum in cycles, 32 per v_mfma_f32_32x32x16_bf16 issued (checked: the round-2
K=2048 twin GEMM counted 1.007e8 = 32 x 6 x 4096 x 1024 x 2048 / 16384);
GRBM_GUI_ACTIVE is the dispatch's busy cycles summed over the 8 XCDs.  So

  busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)

is the fraction of every SIMD's cycles (at the clock the chip actually ran)
in which its matrix core was busy.  It differs from the FLOP-derived fraction
in bench.py's roofline by the clock: that one divides by the 2.4 GHz peak,
this one by the dispatch's own cycles (effective clock = GRBM_GUI_ACTIVE / 8 /
duration, reported too).

On short dispatches GRBM_GUI_ACTIVE over-counts (the implied clock exceeds
the 2.4 GHz peak: MI355X_MICROARCH.md's short-dispatch caveat), so the
GRBM-based quotient is not evidence there.  Every kernel therefore also gets

  busy_at_peak_clock = SQ_VALU_MFMA_BUSY_CYCLES / (1024 x duration x 2.4 GHz)

(the dispatch's own duration from the same pass), a lower bound of the busy
fraction at any clock <= 2.4 GHz, and `busy_fraction` is the GRBM quotient only
where its implied clock is <= 2.4 GHz, else busy_at_peak_clock (`basis` says
which).
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import bench_name  # noqa: E402

N_SIMD, N_XCD = 1024, 8
PEAK_GHZ = 2.4


def main(pmc_dir, config, steps):
    steps = float(steps)
    rows = collections.defaultdict(lambda: collections.defaultdict(dict))
    durations = {}
    for r in csv.DictReader(open(os.path.join(pmc_dir, "run_counter_collection.csv"))):
        key = (bench_name(r["Kernel_Name"]), r.get("Dispatch_Id") or r.get("Correlation_Id"))
        rows[key[0]][key[1]][r["Counter_Name"]] = float(r["Counter_Value"])
        if "End_Timestamp" in r and "Start_Timestamp" in r:
            durations[key] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    out = {"config": config, "source": pmc_dir,
           "formula": "busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 x GRBM_GUI_ACTIVE / 8)",
           "kernels": {}}
    for k, disp in sorted(rows.items()):
        busy = [d["SQ_VALU_MFMA_BUSY_CYCLES"] for d in disp.values()
                if "SQ_VALU_MFMA_BUSY_CYCLES" in d and d.get("GRBM_GUI_ACTIVE")]
        if not busy or sum(busy) == 0:
            continue
        grbm = [d["GRBM_GUI_ACTIVE"] for d in disp.values()
                if "SQ_VALU_MFMA_BUSY_CYCLES" in d and d.get("GRBM_GUI_ACTIVE")]
        n = len(busy)
        mb, gr = sum(busy) / n, sum(grbm) / n
        ent = {"launches": n, "launches_per_step": n / steps,
               "mfma_busy_cycles_per_launch": mb,
               "mfma_32x32x16_equiv_per_launch": mb / 32.0,
               "grbm_gui_active_per_launch": gr,
               "busy_fraction": mb / (N_SIMD * gr / N_XCD)}
        durs = [durations[(k, d)] for d in disp if (k, d) in durations]
        ent["basis"] = "GRBM_GUI_ACTIVE"
        if durs:
            ns = sum(durs) / len(durs)
            ent["avg_duration_us"] = ns / 1e3
            ent["effective_clock_GHz"] = (gr / N_XCD) / ns
            ent["busy_at_peak_clock"] = mb / (N_SIMD * ns * PEAK_GHZ)
            if ent["effective_clock_GHz"] > PEAK_GHZ:
                ent["busy_fraction_grbm"] = ent["busy_fraction"]
                ent["busy_fraction"] = ent["busy_at_peak_clock"]
                ent["basis"] = "duration x 2.4 GHz (GRBM clock above peak)"
        out["kernels"][k] = ent
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(*sys.argv[1:4])
