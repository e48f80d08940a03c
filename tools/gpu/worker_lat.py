"""The reference worker's per-env-step device work (ddpg.py:68-113 with the
fused learner): actor.predict on one state, replay add of one transition,
one learner step with stats.  C2 dims, us per env step (p10 / median / p90)."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
sess, rb, fl, actor = bench.build_learner("c2", 0, 0, 1, 20000)
S, A = 4, 1
rng = np.random.default_rng(0)
st = rng.standard_normal((n + 200, S)).astype(np.float32)


def env_step(i):
    a = actor.predict(st[i:i + 1])
    rb.add(st[i], a[0], 0.5, False, st[i + 1])
    fl.step(stats=True)


for i in range(200):
    env_step(i)
ts = []
for i in range(n):
    t0 = time.perf_counter()
    env_step(i)
    ts.append(1e6 * (time.perf_counter() - t0))
print("env step p10 %.1f median %.1f p90 %.1f us" % tuple(np.percentile(ts, [10, 50, 90])),
      flush=True)
sess.close()
