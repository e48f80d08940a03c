"""Torch-CPU restatement of the reference's learner step.  TEST / BASELINE
INFRASTRUCTURE ONLY: bench.py's `cpu_baseline` leg times it on the host cores
(SURVEY.md §8(d)); the product path never imports it.

The reference runs ddpg.py:86-113 as eight TF 1.3 CPU `sess.run` calls
(TF and the reference cannot run on the GPU box).  This mirrors those calls op
for op in torch eager fp32 on the CPU, without the gRPC hops:

  0 replay_buffer.sample_batch(B)       replay_buffer.py:33-47 (DequeReplay below)
  1 actor.predict_target(s2)            networks.py:82-85
  2 critic.predict_target(s2, a2)       networks.py:183-187
    y = r + gamma * q'  (numpy, ddpg.py:92-97)
  3 critic.train(s, a, y)               networks.py:170-175  fwd + MSE grad + 8 ApplyAdam
  4 actor.predict(s)                    networks.py:77-80
  5 critic.action_gradients(s, a_outs)  networks.py:189-193  (updated critic)
  6 actor.train(s, grads)               networks.py:71-75    fwd recompute + grads + 5 ApplyAdam
  7,8 update_target_network x2          networks.py:87-88, 195-196

Gradients come from torch autograd over the same dataflow TF's gradients
built (grad_ys = -a_gradient for the actor, ones for dQ/da); ApplyAdam is TF's
epsilon-hat form.
"""
import random
from collections import deque

import numpy as np
import torch

from .ddpg_oracle import init_params

F = torch.nn.functional


class DequeReplay:
    """The reference's host replay buffer, restated for the CPU baseline's
    timing (replay_buffer.py:12-47): a bounded deque of per-transition tuples
    (s float64 [S], a float32 [A], r float, t bool, s2 float64 [S]), sampled
    by the stdlib's random.sample over the deque itself (deque indexing is
    O(n/64) per element) and stacked into five arrays with np.array.  This is
    the host cost the reference pays in step 1 of every learner update
    (ddpg.py:88), measured at 0.85 / 2.9 / 46.8 ms for B = 64 / 256 / 4096 on a
    full 1e6 deque."""

    def __init__(self, capacity, seed=1234):
        self.buf = deque(maxlen=int(capacity))
        self.rng = random.Random(seed)

    def fill(self, s, a, r, t, s2):
        """Append rows (row views of the given arrays stand in for the env's
        per-step arrays; np.array stacks views exactly as it stacks copies)."""
        self.buf.extend(zip(list(s), list(a), [float(x) for x in r], [bool(x) for x in t],
                            list(s2)))

    def sample_batch(self, batch_size):
        rows = self.rng.sample(self.buf, batch_size)
        return (np.array([x[0] for x in rows]), np.array([x[1] for x in rows]),
                np.array([x[2] for x in rows]), np.array([x[3] for x in rows]),
                np.array([x[4] for x in rows]))


def _elu(x):
    return torch.where(x < 0, torch.expm1(torch.clamp(x, max=0)), x)


class TorchCPULearner:
    def __init__(self, S, A, H1, H2, scale, seed=1, actor_lr=1e-4, critic_lr=1e-3, tau=1e-3,
                 gamma=0.99):
        a, c = init_params(S, A, H1, H2, seed=seed)
        at, ct = init_params(S, A, H1, H2, seed=seed + 1)
        t = lambda d: {k: torch.tensor(v) for k, v in d.items()}
        self.actor, self.actor_t, self.critic, self.critic_t = t(a), t(at), t(c), t(ct)
        self.scale, self.tau, self.gamma = float(scale), float(tau), float(gamma)
        self.opt = {}
        for name, net, lr in (("actor", self.actor, actor_lr), ("critic", self.critic, critic_lr)):
            self.opt[name] = {"lr": lr, "t": 0,
                              "m": {k: torch.zeros_like(v) for k, v in net.items()},
                              "v": {k: torch.zeros_like(v) for k, v in net.items()}}

    def _actor(self, p, s):
        h1 = _elu(s @ p["W1"] + p["b1"])
        h2 = _elu(h1 @ p["W2"] + p["b2"])
        return torch.tanh(h2 @ p["W3"]) * self.scale

    def _critic(self, p, s, a):
        cat = torch.cat([_elu(s @ p["Ws"] + p["bs"]), _elu(a @ p["Wa"] + p["ba"])], dim=1)
        return _elu(cat @ p["Wh"] + p["bh"]) @ p["Wo"] + p["bo"]

    def _adam(self, name, net, grads, b1=0.9, b2=0.999, eps=1e-8):
        o = self.opt[name]
        o["t"] += 1
        alpha = o["lr"] * np.sqrt(1 - b2 ** o["t"]) / (1 - b1 ** o["t"])
        with torch.no_grad():
            for k, g in grads.items():
                m, v = o["m"][k], o["v"][k]
                m.add_((g - m) * (1 - b1))
                v.add_((g * g - v) * (1 - b2))
                net[k].sub_(m * alpha / (torch.sqrt(v) + eps))

    def _soft(self, net, tgt):
        with torch.no_grad():
            for k in tgt:
                tgt[k].copy_(net[k] * self.tau + tgt[k] * (1.0 - self.tau))

    def step(self, s, a, r, t, s2):
        s, a, s2 = (torch.from_numpy(np.ascontiguousarray(x, np.float32)) for x in (s, a, s2))
        B = s.shape[0]
        with torch.no_grad():                                          # sess.run 1, 2
            q2 = self._critic(self.critic_t, s2, self._actor(self.actor_t, s2)).numpy()
        y = np.where(np.asarray(t)[:, None], np.asarray(r, np.float32)[:, None],
                     np.asarray(r, np.float32)[:, None] + np.float32(self.gamma) * q2)
        y = torch.from_numpy(y.astype(np.float32))
        pc = {k: v.detach().requires_grad_(True) for k, v in self.critic.items()}   # sess.run 3
        q = self._critic(pc, s, a)
        loss = torch.mean((y - q) ** 2)
        gc = torch.autograd.grad(loss, list(pc.values()))
        self._adam("critic", self.critic, dict(zip(pc.keys(), gc)))
        with torch.no_grad():                                          # sess.run 4
            a_outs = self._actor(self.actor, s)
        aa = a_outs.clone().requires_grad_(True)                       # sess.run 5
        qa = self._critic(self.critic, s, aa)
        (da,) = torch.autograd.grad(qa, aa, grad_outputs=torch.ones_like(qa))
        pa = {k: v.detach().requires_grad_(True) for k, v in self.actor.items()}    # sess.run 6
        mu = self._actor(pa, s)
        ga = torch.autograd.grad(mu, list(pa.values()), grad_outputs=-da)
        self._adam("actor", self.actor, dict(zip(pa.keys(), ga)))
        self._soft(self.actor, self.actor_t)                           # sess.run 7, 8
        self._soft(self.critic, self.critic_t)
        return float(loss.detach()), float(q.detach().max()), B
