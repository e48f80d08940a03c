"""C2 (B = 64) synchronous step latency breakdown: host time of the
ddpg_learner_step call alone and call + ddpg_sync, per step (300 steps after
50 warmup).  Run once per DDPG_GRAPH / DDPG_GRAPH_AUTO setting (round 6: a
DDPG_SYNC_SPIN polling variant of ddpg_sync measured equal and was removed)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.getcwd())
import bench  # noqa: E402

sess, rb, fl, _ = bench.build_learner("c2", 0, 0, 1, 100_000)
for _ in range(50):
    fl.step()
    sess.sync()
tc, tt = [], []
for _ in range(300):
    t0 = time.perf_counter()
    fl.step()
    t1 = time.perf_counter()
    sess.sync()
    t2 = time.perf_counter()
    tc.append(1e6 * (t1 - t0))
    tt.append(1e6 * (t2 - t0))
print("%s call median %.1f us p90 %.1f | call+sync median %.1f us p10 %.1f p90 %.1f | steps %s" % (
    sys.argv[1] if len(sys.argv) > 1 else "", np.median(tc), np.percentile(tc, 90), np.median(tt),
    np.percentile(tt, 10), np.percentile(tt, 90), fl.step_counts()), flush=True)
sess.close()
