"""Debug: the bf16 exchange through the proxy communicator, eager or graph
(argv[1] = DDPG_GRAPH_COMM value), small bf16 dims."""
import faulthandler
import os
import sys
faulthandler.enable()
os.environ["DDPG_GRAPH_COMM"] = sys.argv[1]
sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np
from test_gpu_configs import _noisy_params, _open, _rows
from oracle import ddpg_oracle as O
import distributed_ddpg_amd.networks as dd
from distributed_ddpg_amd import _lib
from distributed_ddpg_amd.learner import FusedLearner
from distributed_ddpg_amd.replay_buffer import ReplayBuffer
S, A, H1, H2, scale = 64, 16, 512, 512, 1.0
p = _noisy_params(O, S, A, H1, H2, seed=62, amp=0.02)
rows = _rows(np.random.default_rng(22), 6000, S, A, scale)
sess, actor, critic = _open(dd, O, S, A, H1, H2, scale, p, batch_max=512, world=8, dtype="bf16",
                            critic_lr=0.0)
print("comm init", flush=True)
_lib.check(_lib.lib.ddpg_comm_init_proxy(sess.ctx), sess.ctx)
rb = ReplayBuffer(8000, 77)
rb.add_batch(*rows)
fl = FusedLearner(sess, rb, 4096)
print("step", flush=True)
print(fl.step(stats=True), fl.step_counts(), flush=True)
sess.close()
print("ok", flush=True)
