"""C2 synchronous step latency two ways (ddpg.py:86-113 waits on every
step): fl.step() + sess.sync(), and fl.step(stats=True) (the reference's
sess.run returning Q and loss).  Median / p10 / p90 over n steps, us."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
sess, rb, fl, actor = bench.build_learner(cfg, 0, 0, 1, 100000)
for _ in range(200):
    fl.step()
sess.sync()


def lat(f):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append(1e6 * (time.perf_counter() - t0))
    return "p10 %.1f median %.1f p90 %.1f" % tuple(np.percentile(ts, [10, 50, 90]))


print(cfg, "step+sync   ", lat(lambda: (fl.step(), sess.sync())), flush=True)
print(cfg, "step(stats) ", lat(lambda: fl.step(stats=True)), flush=True)
sess.close()
