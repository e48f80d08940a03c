"""CPU oracle for the DDPG learner-update hot path.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's `cpu_baseline` leg may import
this module, and only as the checker / the CPU baseline -- never as the thing
measured or shipped.  The product path (distributed_ddpg_amd) never imports it.

What it restates (numpy, float64 or float32, op for op):
  * ActorNetwork.create_actor_network       networks.py:51-63
        mu(s) = scale * tanh(elu(elu(s W1 + b1) W2 + b2) W3)       (no last bias)
  * CriticNetwork.create_critic_network     networks.py:147-162
        Q(s,a) = elu([elu(s Ws + bs) | elu(a Wa + ba)] Wh + bh) Wo + bo
  * CriticNetwork loss/optimizer + train    networks.py:130-137, 170-175
        L = mean((y - Q)^2), Adam(lr_c); returns [Q_pre_update, None, L]
  * CriticNetwork.action_grads              networks.py:143, 189-193
  * ActorNetwork.actor_gradients/train      networks.py:39-47, 71-75
        g = tf.gradients(mu, theta, -dQ/da)   (a batch SUM, no 1/B)
  * update_target_network_params            networks.py:34-37, 126-128
        theta' <- theta*tau + theta'*(1-tau)  (fp32 consts 0.001 / 0.999)
  * TD target                               ddpg.py:90-100
  * learner step orchestration              ddpg.py:86-113
  * init-time soft blend of targets         ddpg.py:224-229
TF 1.3 kernel semantics (third-party, not vendored; constants confirmed in
InvertedPendulum/model_ddpg/model-1410.meta -> tests/golden/meta_constants.json):
  * Elu(x) = x<0 ? exp(x)-1 : x;  EluGrad(dy, y) = y<0 ? dy*(y+1) : dy
  * TanhGrad(y, dy) = dy*(1-y*y)
  * ApplyAdam: alpha = lr*sqrt(1-b2^t)/(1-b1^t); m += (g-m)(1-b1);
               v += (g*g-v)(1-b2); var -= m*alpha/(sqrt(v)+eps);
    beta powers start at b1/b2 and are multiplied by b1/b2 after the update.
  * MSE grad: dQ = -(2*(y-Q)) / B   (Mean_grad 1/B, Square_grad 2x, Sub -1)

Parity status: TF 1.3 / tflearn / gym are not installed, so the reference's
own graphs are executed instead: tests/golden/tfgraph.py interprets the
MetaGraphDefs the reference saved (InvertedPendulum model-1410.meta,
MountainCar model-120.meta) node by node from their checkpoints, and
tests/test_graph_pin.py holds this restatement to those trajectories at 1e-6
(graph_ip1410.npz; graph_ip1410_fresh.npz with the graph's own optimizer
initializers, i.e. Adam bias correction; graph_mc120.npz with the MountainCar
widths and a fitted scaler).  Also: an independent torch-fp64 autograd
formulation and finite differences (tests/test_oracle.py), the decoded
checkpoints (tests/golden/*.npz) and the graph constants (meta_constants.json).
"""
import numpy as np

ACTOR_KEYS = ("W1", "b1", "W2", "b2", "W3")
CRITIC_KEYS = ("Ws", "bs", "Wa", "ba", "Wh", "bh", "Wo", "bo")

# tf.trainable_variables() order == checkpoint tensor names
CKPT_ACTOR = ("FullyConnected/W", "FullyConnected/b", "FullyConnected_1/W",
              "FullyConnected_1/b", "FullyConnected_2/W")
CKPT_ACTOR_T = ("FullyConnected_3/W", "FullyConnected_3/b", "FullyConnected_4/W",
                "FullyConnected_4/b", "FullyConnected_5/W")
CKPT_CRITIC = ("FullyConnected_6/W", "FullyConnected_6/b", "FullyConnected_7/W",
               "FullyConnected_7/b", "FullyConnected_8/W", "FullyConnected_8/b",
               "FullyConnected_9/W", "FullyConnected_9/b")
CKPT_CRITIC_T = ("FullyConnected_10/W", "FullyConnected_10/b", "FullyConnected_11/W",
                 "FullyConnected_11/b", "FullyConnected_12/W", "FullyConnected_12/b",
                 "FullyConnected_13/W", "FullyConnected_13/b")


def actor_shapes(S, A, H1, H2):
    return {"W1": (S, H1), "b1": (H1,), "W2": (H1, H2), "b2": (H2,), "W3": (H2, A)}


def critic_shapes(S, A, H1, H2):
    return {"Ws": (S, H1), "bs": (H1,), "Wa": (A, H1), "ba": (H1,),
            "Wh": (2 * H1, H2), "bh": (H2,), "Wo": (H2, 1), "bo": (1,)}


# ---------------------------------------------------------------- TF kernels
def elu(x):
    """TF 1.3 Elu: (x < 0).select(exp(x) - 1, x)."""
    one = x.dtype.type(1)
    return np.where(x < 0, np.exp(np.minimum(x, 0)) - one, x)


def elu_grad(dy, y):
    """TF 1.3 EluGrad computed from the OUTPUT y."""
    one = y.dtype.type(1)
    return np.where(y < 0, dy * (y + one), dy)


def tanh_grad(y, dy):
    one = y.dtype.type(1)
    return dy * (one - y * y)


def dense(x, W, b=None):
    z = x @ W
    if b is not None:
        z = z + b
    return z


# ---------------------------------------------------------------- forward
def actor_forward(p, s, scale):
    """networks.py:51-63.  Returns (h1, h2, o, mu) with o = tanh(.)."""
    dt = s.dtype.type
    h1 = elu(dense(s, p["W1"], p["b1"]))
    h2 = elu(dense(h1, p["W2"], p["b2"]))
    o = np.tanh(h2 @ p["W3"])
    return h1, h2, o, o * dt(scale)


def critic_forward(p, s, a):
    """networks.py:147-162.  Returns (cs, ca, h, q)."""
    cs = elu(dense(s, p["Ws"], p["bs"]))
    ca = elu(dense(a, p["Wa"], p["ba"]))
    cat = np.concatenate([cs, ca], axis=1)
    h = elu(dense(cat, p["Wh"], p["bh"]))
    q = dense(h, p["Wo"], p["bo"])
    return cs, ca, h, q


# ---------------------------------------------------------------- backward
def critic_grads(p, s, a, dq):
    """Gradients of sum(dq * Q(s,a)) wrt critic params and wrt a."""
    cs, ca, h, q = critic_forward(p, s, a)
    H1 = cs.shape[1]
    cat = np.concatenate([cs, ca], axis=1)
    g = {}
    g["Wo"] = h.T @ dq
    g["bo"] = dq.sum(axis=0)
    dh = elu_grad(dq @ p["Wo"].T, h)
    g["Wh"] = cat.T @ dh
    g["bh"] = dh.sum(axis=0)
    dcat = dh @ p["Wh"].T
    dcs = elu_grad(dcat[:, :H1], cs)
    dca = elu_grad(dcat[:, H1:], ca)
    g["Ws"] = s.T @ dcs
    g["bs"] = dcs.sum(axis=0)
    g["Wa"] = a.T @ dca
    g["ba"] = dca.sum(axis=0)
    da = dca @ p["Wa"].T
    return g, da, q


def critic_action_grads(p, s, a):
    """networks.py:143 -- tf.gradients(out, action) with grad_ys = 1."""
    dq = np.ones((s.shape[0], 1), dtype=s.dtype)
    _, da, _ = critic_grads(p, s, a, dq)
    return da


def actor_grads(p, s, a_gradient, scale):
    """networks.py:44 -- tf.gradients(scaled_out, params, -a_gradient)."""
    dt = s.dtype.type
    h1, h2, o, _ = actor_forward(p, s, scale)
    dmu = -a_gradient
    dz3 = tanh_grad(o, dmu * dt(scale))
    g = {"W3": h2.T @ dz3}
    dz2 = elu_grad(dz3 @ p["W3"].T, h2)
    g["W2"] = h1.T @ dz2
    g["b2"] = dz2.sum(axis=0)
    dz1 = elu_grad(dz2 @ p["W2"].T, h1)
    g["W1"] = s.T @ dz1
    g["b1"] = dz1.sum(axis=0)
    return g


def mse_loss_and_grad(y, q):
    """tflearn.mean_square(y, out) = mean(square(y - out)); d/dout."""
    dt = q.dtype.type
    B = q.shape[0]
    diff = y - q
    loss = np.mean(np.square(diff), dtype=q.dtype)
    dq = -((dt(1) / dt(B)) * (dt(2) * diff))
    return loss, dq


# ---------------------------------------------------------------- optimizer
class TFAdam:
    """tf.train.AdamOptimizer(lr) with TF 1.3 ApplyAdam semantics, one
    instance per network (own beta1_power / beta2_power, as in the graph)."""

    def __init__(self, shapes, lr, dtype, beta1=0.9, beta2=0.999, eps=1e-8):
        dt = np.dtype(dtype).type
        self.dt = dt
        # the graph's constants are float32 (Adam/learning_rate, Adam/beta1, ...
        # in model-1410.meta); a float64 run widens those float32 values
        self.lr, self.b1, self.b2, self.eps = (dt(np.float32(x)) for x in (lr, beta1, beta2, eps))
        self.m = {k: np.zeros(s, dtype) for k, s in shapes.items()}
        self.v = {k: np.zeros(s, dtype) for k, s in shapes.items()}
        self.b1p = self.b1
        self.b2p = self.b2

    def alpha(self):
        one = self.dt(1)
        return self.lr * np.sqrt(one - self.b2p) / (one - self.b1p)

    def apply(self, params, grads):
        one = self.dt(1)
        alpha = self.alpha()
        for k, g in grads.items():
            m, v = self.m[k], self.v[k]
            m += (g - m) * (one - self.b1)
            v += (g * g - v) * (one - self.b2)
            params[k] = params[k] - (m * alpha) / (np.sqrt(v) + self.eps)
        self.b1p = self.b1p * self.b1
        self.b2p = self.b2p * self.b2


def soft_update(online, target, tau):
    """networks.py:34-37: target.assign(theta*tau + theta'*(1.-tau))."""
    for k in target:
        dt = target[k].dtype.type  # float32 graph constants Mul_2/y, Mul_3/y
        target[k] = online[k] * dt(np.float32(tau)) + target[k] * dt(np.float32(1.0 - tau))


def td_target(r, t, q2, gamma):
    """ddpg.py:92-100 vectorised: y = r if t else r + gamma*q'.  Computed at
    q2's precision (the 2017 numpy semantics: fl(fl(r) + fl(gamma*q')), with
    the Python-float gamma cast to the float32 array's type)."""
    dt = q2.dtype.type
    r = r.astype(q2.dtype).reshape(-1, 1)
    t = t.astype(bool).reshape(-1, 1)
    return np.where(t, r, r + dt(np.float32(gamma)) * q2)  # GAMMA * f32 array -> f32 GAMMA


# ---------------------------------------------------------------- init
def init_params(S, A, H1, H2, seed, dtype=np.float32):
    """tflearn defaults (networks.py:54-59,151-161; constants in .meta):
    W ~ TruncatedNormal(0, 0.02) (re-draw beyond 2 sigma), b = 0, last-layer
    W ~ U(-3e-3, 3e-3).  TF's Philox streams cannot be reproduced, so this is a
    seeded numpy stand-in; parity runs inject weights instead."""
    rng = np.random.default_rng(seed)

    def tn(shape):
        x = rng.standard_normal(shape)
        bad = np.abs(x) > 2.0
        while bad.any():
            x[bad] = rng.standard_normal(int(bad.sum()))
            bad = np.abs(x) > 2.0
        return (0.02 * x).astype(dtype)

    def un(shape):
        return rng.uniform(-0.003, 0.003, shape).astype(dtype)

    def z(shape):
        return np.zeros(shape, dtype)

    actor = {"W1": tn((S, H1)), "b1": z(H1), "W2": tn((H1, H2)), "b2": z(H2),
             "W3": un((H2, A))}
    critic = {"Ws": tn((S, H1)), "bs": z(H1), "Wa": tn((A, H1)), "ba": z(H1),
              "Wh": tn((2 * H1, H2)), "bh": z(H2), "Wo": un((H2, 1)), "bo": z(1)}
    return actor, critic


# ---------------------------------------------------------------- learner
class Learner:
    """One worker's learner state + the reference's learner step.

    `step(batch)` follows ddpg.py:86-113 exactly (same call order, the
    critic's action gradient taken with the already-updated critic, targets
    blended after both trains).  `recompute_actor_forward=True` recomputes the
    actor forward inside actor.train as TF does (cost only; same numbers)."""

    def __init__(self, S, A, H1, H2, scale, actor_lr=1e-4, critic_lr=1e-3, tau=1e-3,
                 gamma=0.99, dtype=np.float64, params=None, init_blend=True, CH1=None, CH2=None):
        self.S, self.A, self.H1, self.H2 = S, A, H1, H2
        CH1, CH2 = CH1 or H1, CH2 or H2
        self.scale, self.tau, self.gamma = scale, tau, gamma
        self.dtype = np.dtype(dtype)
        if params is None:
            raise ValueError("pass params={'actor','actor_t','critic','critic_t'}")
        cv = lambda d: {k: np.array(v, dtype=self.dtype) for k, v in d.items()}
        self.actor, self.actor_t = cv(params["actor"]), cv(params["actor_t"])
        self.critic, self.critic_t = cv(params["critic"]), cv(params["critic_t"])
        self.actor_opt = TFAdam(actor_shapes(S, A, H1, H2), actor_lr, self.dtype)
        self.critic_opt = TFAdam(critic_shapes(S, A, CH1, CH2), critic_lr, self.dtype)
        if init_blend:  # ddpg.py:224-229
            soft_update(self.actor, self.actor_t, tau)
            soft_update(self.critic, self.critic_t, tau)

    # --- networks.py session wrappers
    def actor_predict(self, s, target=False):
        return actor_forward(self.actor_t if target else self.actor, s, self.scale)[3]

    def critic_predict(self, s, a, target=False):
        return critic_forward(self.critic_t if target else self.critic, s, a)[3]

    def critic_train(self, s, a, y):
        q = critic_forward(self.critic, s, a)[3]
        loss, dq = mse_loss_and_grad(y, q)
        g, _, _ = critic_grads(self.critic, s, a, dq)
        self.critic_opt.apply(self.critic, g)
        return q, loss, g

    def action_gradients(self, s, a):
        return critic_action_grads(self.critic, s, a)

    def actor_train(self, s, a_gradient):
        g = actor_grads(self.actor, s, a_gradient, self.scale)
        self.actor_opt.apply(self.actor, g)
        return g

    def update_targets(self):
        soft_update(self.actor, self.actor_t, self.tau)
        soft_update(self.critic, self.critic_t, self.tau)

    def step(self, s, a, r, t, s2):
        """ddpg.py:86-113 on an already-sampled batch (fp32/fp64 arrays)."""
        dt = self.dtype
        s, a, s2 = (np.asarray(x, dt) for x in (s, a, s2))
        target_q = self.critic_predict(s2, self.actor_predict(s2, True), True)
        y = td_target(np.asarray(r), np.asarray(t), target_q, self.gamma)
        q, loss, gc = self.critic_train(s, a, y)
        a_outs = self.actor_predict(s)
        da = self.action_gradients(s, a_outs)
        ga = self.actor_train(s, da)
        self.update_targets()
        return {"q": q, "loss": loss, "y": y, "a_outs": a_outs, "da": da,
                "critic_grads": gc, "actor_grads": ga}

    def state(self):
        return {"actor": self.actor, "actor_t": self.actor_t, "critic": self.critic,
                "critic_t": self.critic_t}


def flops_per_step(S, A, H1, H2, B, tf_recompute=False, survey=False):
    """Algorithmic FLOP of one fused learner step.

    Default (minimal) count, MAC per sample:
      3*AF (target fwd, online fwd, weight grads) + 4*CF (target fwd, train fwd,
      weight grads, action-grad fwd) + critic dX (H2 + 2*H1*H2)
      + action-grad dX (H2 + H1*H2 + A*H1; only the action half of dcat is
      needed) + actor dX (H2*A + H1*H2) + dQ head (H2).
    survey=True reproduces SURVEY.md §8(d)'s count, which charges the full
    2*H1*H2 for the action-grad dX (+H1*H2 - H2 per sample)."""
    AF = S * H1 + H1 * H2 + H2 * A
    CF = S * H1 + A * H1 + 2 * H1 * H2 + H2
    if survey:
        dX = 2 * (H2 + 2 * H1 * H2) + A * H1 + H2 * A + H1 * H2
    else:
        dX = 3 * H2 + 4 * H1 * H2 + A * H1 + H2 * A
    mac = 3 * AF + 4 * CF + dX
    if tf_recompute:
        mac += AF
    return 2 * B * mac
