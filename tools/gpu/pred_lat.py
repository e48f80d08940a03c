"""Action-selection latency breakdown (ddpg.py:68-70): actor.predict on one
state vs the bare C-ABI call with preallocated buffers, C2 InvertedPendulum
dims.  Prints one line per form (us per call)."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import distributed_ddpg_amd.networks as nets  # noqa: E402
from distributed_ddpg_amd import _lib  # noqa: E402

S, A, H1, H2 = 4, 1, 128, 200
nets.reset_default_graph()
actor = nets.ActorNetwork(S, A, 3.0, 1e-4, 1e-3, None, h1=H1, h2=H2)
critic = nets.CriticNetwork(S, A, 1e-3, 1e-3, 10, None, h1=H1, h2=H2)
sess = nets.Session(batch_max=64)
sess.run(nets.global_variables_initializer(seed=1))
actor.set_session(sess)
critic.set_session(sess)
s = np.random.default_rng(0).standard_normal((1, S)).astype(np.float32)
out = np.empty((1, A), np.float32)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000


def timeit(f):
    for _ in range(100):
        f()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    return 1e6 * (time.perf_counter() - t0) / n


print("predict %.2f us" % timeit(lambda: actor.predict(s)), flush=True)
ps, po = _lib.fptr(s), _lib.fptr(out)
print("c_abi   %.2f us" % timeit(lambda: _lib.lib.ddpg_actor_forward(sess.ctx, 0, ps, 1, po)),
      flush=True)
sess.close()
