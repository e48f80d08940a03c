"""Summarise a rocprofv3 rocpd database (results.db) into the committed text
form: per-kernel totals (== `rocprofv3 --stats`) and per-grid GEMM detail.

  python profiles/summarize.py gpurun_out/prof_r1/run_results.db > profiles/r1_c3_kernels.txt
"""
import sqlite3
import sys


def main(path):
    db = sqlite3.connect(path)
    cur = db.cursor()
    print("# rocprofv3 --kernel-trace --stats summary of %s" % path)
    print("# name | calls | total_us | avg_us | pct")
    for name, calls, tot, avg, pct in cur.execute(
            "select name, total_calls, total_duration, average, percentage from top_kernels"):
        print("%s | %d | %.1f | %.3f | %.2f" % (name, calls, tot, avg, pct))
    print()
    print("# per-grid detail: name | grid(blocks x,y,z) | calls | avg_us | vgpr | lds")
    q = ("select name, grid_x/workgroup_x, grid_y/workgroup_y, grid_z/workgroup_z, count(*), "
         "avg(duration)/1000.0, vgpr_count, lds_size from kernels group by name, grid_x, grid_y, "
         "grid_z order by sum(duration) desc")
    for r in cur.execute(q):
        print("%s | %dx%dx%d | %d | %.2f | %d | %d" % r)


if __name__ == "__main__":
    main(sys.argv[1])
