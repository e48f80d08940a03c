"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

  python profiles/pmc_traffic.py <fetch_dir> <write_dir> <config> <steps> > profiles/rN_pmc_<config>.json

<steps> = fused learner steps the profiled command ran (warmup + steps + the
bench's latency and profile passes); launches_per_step lets bench.py refuse a
pass whose launch set does not match the run it reports.

Each pass is its own run of the same bench command (FETCH_SIZE takes 3 of the 4
TCC slots, WRITE_SIZE 2, so they cannot share one pass), e.g.

  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
      -d gpurun_out/pmc_fetch -o run -- python3 bench.py --no-cpu --no-small ...

Corrections (MI355X_MICROARCH.md, HBM section): rocprofv3 reports both counters in
KB; on gfx950 FETCH_SIZE counts 128-B requests at 64 B, i.e. exactly half the bytes
of a wide coalesced streaming read, so it is doubled; WRITE_SIZE is exact for
16-B-per-lane streaming stores.  Infinity-Cache hits are counted as fetches.
bench.py reads the JSON this writes and reports traffic = corrected fetch + write
bytes per launch of the dominant kernel.
"""
import collections
import csv
import json
import os
import re
import sys


def bench_name(rocprof_name):
    """'void ddpg::gemm_f32_kernel<0, 1, 4, 4, 64, 64>(ddpg::GemmArgs)' -> bench key."""
    m = re.search(r"ddpg::(\w+)(?:<([^>]*)>)?\(", rocprof_name)
    if not m:
        return rocprof_name
    sym, targs = m.group(1), m.group(2)
    if targs is None:
        return sym
    a = [x.strip() for x in targs.split(",")]
    if sym == "thin_k_kernel" and len(a) <= 2:  # MODE (generic / forward / backward form), DW
        return {"0": "thin_k_kernel", "1": "thin_k_kernel<FWD>", "2": "thin_k_kernel<BWD>"}.get(
            a[0], "thin_k_kernel<%s>" % a[0])
    if len(a) < 2:
        return "%s<%s>" % (sym, a[0])
    lay = {"0": "RK", "1": "KR"}
    a[0], a[1] = lay.get(a[0], a[0]), lay.get(a[1], a[1])
    if sym == "gemm_h16i_pack_kernel" and len(a) == 2:
        return "%s<%s,%s,NP=1>" % (sym, a[0], a[1])
    if sym == "gemm_h3m_pack_kernel" and len(a) == 2:
        return "%s<%s,%s,NP=3>" % (sym, a[0], a[1])
    if sym in ("gemm_hw_kernel", "gemm_hw_pack_kernel"):  # bf16 (one plane) by construction
        return "%s<%s,%s,NP=1>" % (sym, a[0], a[1])
    if sym == "gemm_s3_kernel" and len(a) == 3:
        # bench.py labels the one-plane instantiation gemm_bf16_kernel
        return "%s<%s,%s>" % ("gemm_s3_kernel" if a[2] == "3" else "gemm_bf16_kernel", a[0], a[1])
    if sym in ("gemm_h_kernel", "gemm_h16_kernel") and len(a) >= 3:
        # bench.py labels it by operand layouts and plane count
        return "%s<%s,%s,NP=%s>" % (sym, a[0], a[1], a[2])
    if sym in ("gemm_h3_kernel", "gemm_h3m_kernel") and len(a) == 2:  # three planes by construction
        return "%s<%s,%s,NP=3>" % (sym, a[0], a[1])
    if sym == "gemm_h16i_kernel" and len(a) == 2:  # one plane by construction
        return "%s<%s,%s,NP=1>" % (sym, a[0], a[1])
    if sym == "gemm_h256_kernel" and len(a) == 3:
        return "%s<%s,%s,MODE=%s>" % (sym, a[0], a[1], a[2])
    return "%s<%s>" % (sym, ",".join(a))


def load(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(path, "run_counter_collection.csv"))):
        if r["Counter_Name"] == counter:
            agg[bench_name(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
    return agg


def main(fetch_dir, write_dir, config, steps):
    steps = float(steps)
    f, w = load(fetch_dir, "FETCH_SIZE"), load(write_dir, "WRITE_SIZE")
    out = {"config": config, "source": [fetch_dir, write_dir],
           "correction": "fetch_bytes = 2 x FETCH_SIZE (gfx950 half-count of 128-B requests); "
                         "write_bytes = WRITE_SIZE; KB -> B x 1024",
           "kernels": {}}
    for k in sorted(set(f) | set(w)):
        fb = sum(f.get(k, [0.0])) / max(1, len(f.get(k, [])))
        wb = sum(w.get(k, [0.0])) / max(1, len(w.get(k, [])))
        out["kernels"][k] = {"launches": len(f.get(k, [])),
                             "launches_per_step": len(f.get(k, [])) / steps,
                             "fetch_size_raw_per_launch": fb,
                             "fetch_bytes_per_launch": 2.0 * fb,
                             "write_bytes_per_launch": wb,
                             "traffic_bytes_per_launch": 2.0 * fb + wb}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(*sys.argv[1:5])
