"""GPU box: host-side cost of one fused learner step call (C2 / C3), graph vs
eager: time N calls without synchronising (host issue rate), then the total
once the stream drains.  Diagnostic only."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 500
torch.cuda.set_device(0)
sess, rb, fl, _ = bench.build_learner(cfg, 0, 0, 1, 200000)
for _ in range(20):
    fl.step()
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    for _ in range(N):
        fl.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("%s graph=%s: host issue %.1f us/call, total %.1f us/step" %
          (cfg, os.environ.get("DDPG_GRAPH", "1"), 1e6 * (t1 - t0) / N, 1e6 * (t2 - t0) / N),
          flush=True)
# the sampler alone
import ctypes  # noqa: E402
sess.close()
