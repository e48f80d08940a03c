"""Diagnostic (GPU box): determinism of one bf16 fused step at the 1024-wide
config under the default plan and DDPG_GEMM256=1, per gradient tensor."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import distributed_ddpg_amd.networks as dd  # noqa: E402
from oracle import ddpg_oracle as O  # noqa: E402
from test_gpu_parity import _params, normrel  # noqa: E402
from test_gpu_switches import _run  # noqa: E402

p, _ = _params(O, "wide")
runs = {}
for tag, env in (("d1", {}), ("d2", {}), ("g1", {"DDPG_GEMM256": "1"}), ("g2", {"DDPG_GEMM256": "1"}),
                 ("k1", {"DDPG_KCOMB": "0"}), ("k2", {"DDPG_KCOMB": "0"})):
    for k in ("DDPG_GEMM256", "DDPG_KCOMB"):
        os.environ.pop(k, None)
    os.environ.update(env)
    runs[tag] = _run(dd, O, "wide", p, 1, dtype="bf16")
names = ["actor_grad", "critic_grad"]
for a, b in (("d1", "d2"), ("g1", "g2"), ("k1", "k2"), ("d1", "g1"), ("d1", "k1")):
    out = []
    for i, nm in zip((8, 9), names):
        out.append("%s %s" % (nm, ["%.2e" % normrel(v, u) for u, v in zip(runs[a]["state"][i],
                                                                          runs[b]["state"][i])]))
    print(a, b, "; ".join(out), flush=True)
