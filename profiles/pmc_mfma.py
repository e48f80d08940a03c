"""Per-kernel MFMA busy fraction from one rocprofv3 PMC pass.

  python profiles/pmc_mfma.py <pmc_dir> <config> <steps> > profiles/rN/mfma_<config>.json

The pass (tools/gpu/profile.sh) collects SQ_VALU_MFMA_BUSY_CYCLES,
SQ_WAVE_CYCLES, SQ_WAVES and GRBM_GUI_ACTIVE for every dispatch of the bench
command.  Units (MI355X_MICROARCH.md cycle-constants table):
SQ_VALU_MFMA_BUSY_CYCLES is a device sum in cycles (32 per
v_mfma_f32_32x32x16_bf16; checked: the round-2 K=2048 twin GEMM counted
1.007e8 = 32 x 6 x 4096 x 1024 x 2048 / 16384); SQ_WAVE_CYCLES counts
quad-cycles of wave lifetime.

Per kernel (dispatch averages, duration D from the same pass):
  busy_at_peak_clock = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x D x 2.4 GHz)
                       -- a lower bound of the busy fraction at any clock
  wave_clock_GHz     = 4 SQ_WAVE_CYCLES / SQ_WAVES / D -- a lower bound of
                       the shader clock (a wave lives at most D), tight for
                       one-round grids whose waves span the dispatch
  busy_at_wave_clock = SQ_VALU_MFMA_BUSY_CYCLES / (1024 x D x wave clock)
                       -- an upper bound (round 6)
GRBM_GUI_ACTIVE / 8 / D is reported as `grbm_clock_GHz` only: it reads above
the shader clock on dispatches shorter than ~0.3 ms (MI355X_MICROARCH.md
'DVFS give-back'), i.e. on every kernel of the step, so it is no clock
measurement here (rounds 3-5 used it; round 6 dropped it).  `busy_fraction`
= busy_at_peak_clock (the conservative figure bench.py sums).
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
           "formula": "busy_at_peak_clock = SQ_VALU_MFMA_BUSY_CYCLES / (1024 x D x 2.4 GHz); "
                      "busy_at_wave_clock with wave clock = 4 SQ_WAVE_CYCLES / SQ_WAVES / D",
           "kernels": {}}
    for k, disp in sorted(rows.items()):
        ds = [(d, i) for i, d in disp.items() if d.get("SQ_VALU_MFMA_BUSY_CYCLES")]
        if not ds:
            continue
        n = len(ds)
        avg = lambda c: sum(d.get(c, 0.0) for d, _ in ds) / n
        mb = avg("SQ_VALU_MFMA_BUSY_CYCLES")
        ent = {"launches": n, "launches_per_step": n / steps,
               "mfma_busy_cycles_per_launch": mb,
               "mfma_32x32x16_equiv_per_launch": mb / 32.0}
        durs = [durations[(k, i)] for _, i in ds if (k, i) in durations]
        if durs:
            ns = sum(durs) / len(durs)
            ent["avg_duration_us"] = ns / 1e3
            ent["busy_at_peak_clock"] = mb / (N_SIMD * ns * PEAK_GHZ)
            ent["busy_fraction"] = ent["busy_at_peak_clock"]
            waves = avg("SQ_WAVES")
            if waves:
                wc = 4.0 * avg("SQ_WAVE_CYCLES") / waves / ns
                ent["wave_clock_GHz"] = wc
                ent["busy_at_wave_clock"] = mb / (N_SIMD * ns * wc) if wc else None
            if avg("GRBM_GUI_ACTIVE"):
                ent["grbm_clock_GHz"] = avg("GRBM_GUI_ACTIVE") / N_XCD / ns
        out["kernels"][k] = ent
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(*sys.argv[1:4])
