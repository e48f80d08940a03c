"""The reference's per-step sequence through the 1:1 methods (ddpg.py:86-113:
target Q, critic.train, actor.predict, action_gradients, actor.train, both
soft updates) at C2 dims, B = 64: wall time per step, us (median / p10 / p90)."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import distributed_ddpg_amd.networks as nets  # noqa: E402

S, A, H1, H2, B = 4, 1, 128, 200, 64
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
nets.reset_default_graph()
actor = nets.ActorNetwork(S, A, 3.0, 1e-4, 1e-3, None, h1=H1, h2=H2)
critic = nets.CriticNetwork(S, A, 1e-3, 1e-3, 10, None, h1=H1, h2=H2)
sess = nets.Session(batch_max=B)
sess.run(nets.global_variables_initializer(seed=1))
actor.set_session(sess)
critic.set_session(sess)
rng = np.random.default_rng(0)
s = rng.standard_normal((B, S)).astype(np.float32)
a = rng.uniform(-3, 3, (B, A)).astype(np.float32)
r = rng.standard_normal(B).astype(np.float32)
t = rng.random(B) < 0.05
s2 = rng.standard_normal((B, S)).astype(np.float32)


def step():
    tq = critic.predict_target(s2, actor.predict_target(s2))
    y = np.where(t, r, r + 0.99 * tq[:, 0]).astype(np.float32)[:, None]
    critic.train(s, a, y)
    mu = actor.predict(s)
    g = critic.action_gradients(s, mu)
    actor.train(s, g[0])
    actor.update_target_network()
    critic.update_target_network()


for _ in range(100):
    step()
ts = []
for _ in range(n):
    t0 = time.perf_counter()
    step()
    ts.append(1e6 * (time.perf_counter() - t0))
print("1:1 step p10 %.1f median %.1f p90 %.1f us" % tuple(np.percentile(ts, [10, 50, 90])), flush=True)
sess.close()
