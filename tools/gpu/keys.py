"""Per-key in-step kernel times with shapes (DDPG_PROF_SHAPES=1): one config,
warm-up steps, then profiled steps; prints ms per step by key, largest first.
  python tools/gpu/keys.py c5 [steps]"""
import os
import sys

os.environ["DDPG_PROF_SHAPES"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
from distributed_ddpg_amd.learner import Profile  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dtype = "bf16" if cfg == "c5" else "fp32"
sess, rb, fl, _ = bench.build_learner(cfg, 0, 0, 1, 200_000, dtype=dtype)
for _ in range(5):
    fl.step()
torch.cuda.synchronize()
prof = Profile(sess)
prof.enable(True)
for _ in range(steps):
    fl.step()
torch.cuda.synchronize()
keys = prof.read(128)
prof.enable(False)
tot = 0.0
for k, v in sorted(keys.items(), key=lambda kv: -kv[1]["ms"]):
    per = v["ms"] / steps
    tot += per
    print("%-70s %7.1f us/step  %5.2f launches/step  %7.2f us avg" %
          (k, 1e3 * per, v["launches"] / steps, 1e3 * v["ms"] / max(1, v["launches"])))
print("sum %.1f us/step" % (1e3 * tot))
