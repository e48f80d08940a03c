"""ActorNetwork / CriticNetwork with the reference's interface (networks.py),
computed by the HIP kernels of libddpg_hip.so.

Drop-in surface (reference networks.py):
  ActorNetwork(state_dim, action_dim, action_scale, learning_rate, tau, scaler)  :17
      predict / predict_target / train / update_target_network
      get_num_trainable_vars / restore_params / set_session                    :71-99
  CriticNetwork(state_dim, action_dim, learning_rate, tau, num_actor_vars, scaler) :109
      train -> [Q_pre_update, None, loss] / predict / predict_target
      action_gradients -> [dQ/da] / update_target_network / ...               :170-207
The TF graph + tf.Session pair is replaced by a `Session` owning one
ddpg_ctx (device weights, Adam state, workspaces) built from the networks
registered on the default `Graph`, exactly as the reference builds both
networks on TF's default graph and then opens a session on it (ddpg.py:202-239).

Hidden widths default to the reference's 128/200 (networks.py:54-55,151-156)
and may be overridden (h1=, h2=) for the synthetic configurations.
Inputs are numpy arrays; the scaler (sklearn-style .transform) is applied in
float64 on the host and the result fed as float32, as TF's feed_dict does.
"""
import numpy as np

from . import _lib
from ._lib import check, f32, fptr, lib


class Graph:
    """Stand-in for TF's default graph: the networks built so far."""

    def __init__(self):
        self.actor = None
        self.critic = None


_default_graph = Graph()


def get_default_graph():
    return _default_graph


def reset_default_graph():
    global _default_graph
    _default_graph = Graph()
    return _default_graph


class _InitOp:
    """tf.global_variables_initializer() stand-in (ddpg.py:208, :238)."""

    def __init__(self, seed):
        self.seed = seed


def global_variables_initializer(seed=1234):
    return _InitOp(seed)


class Session:
    """tf.Session stand-in owning one device context (one per process/GPU).

    Session(target=None, graph=None, device=0, batch_max=4096, rank=0, world=1)
    `target` (the reference's server.target) is accepted and ignored.
    """

    def __init__(self, target=None, graph=None, device=0, batch_max=4096, rank=0, world=1,
                 dtype="fp32"):
        g = graph or _default_graph
        if g.actor is None or g.critic is None:
            raise ValueError("build ActorNetwork and CriticNetwork before opening a Session")
        a, c = g.actor, g.critic
        if (a.s_dim, a.a_dim) != (c.s_dim, c.a_dim):
            raise ValueError("actor/critic dims differ")
        self.actor, self.critic = a, c
        self.batch_max = int(batch_max)
        cfg = _lib.Cfg()
        cfg.state_dim, cfg.action_dim = a.s_dim, a.a_dim
        cfg.h1, cfg.h2 = a.h1, a.h2
        cfg.critic_h1, cfg.critic_h2 = c.h1, c.h2
        cfg.batch_max = self.batch_max
        cfg.actor_lr, cfg.critic_lr = a.learning_rate, c.learning_rate
        if a.tau != c.tau:
            raise ValueError("actor and critic tau differ")
        cfg.tau = a.tau
        cfg.gamma = 0.99
        cfg.action_scale = float(a.action_scale)
        cfg.beta1, cfg.beta2, cfg.epsilon = 0.9, 0.999, 1e-8
        cfg.dtype = {"fp32": _lib.FP32, "bf16": _lib.BF16}[dtype]
        cfg.device, cfg.rank, cfg.world = int(device), int(rank), int(world)
        self.cfg = cfg
        self.ctx = _lib.ctypes.c_void_p()
        check(lib.ddpg_create(_lib.ctypes.byref(cfg), _lib.ctypes.byref(self.ctx)))
        # action selection's host staging: ctypes arrays passed as they are
        # (numpy's .ctypes pointer conversion costs microseconds per call)
        self._io_in = (_lib.ctypes.c_float * _IO_FLOATS)()
        self._io_out = (_lib.ctypes.c_float * _IO_FLOATS)()
        self._io_in_np = np.frombuffer(self._io_in, np.float32)
        self._io_out_np = np.frombuffer(self._io_out, np.float32)

    # --- tf.Session-like
    def run(self, fetches, feed_dict=None):
        if isinstance(fetches, _InitOp):
            self.initialize(fetches.seed)
            return None
        if isinstance(fetches, (list, tuple)):
            return [self.run(f, feed_dict) for f in fetches]
        raise TypeError("Session.run supports the variables initializer only; call the "
                        "network methods instead")

    def initialize(self, seed=1234):
        """Independent tflearn-style draws for online and target networks
        (networks.py:30,122 build targets with their own initialisers)."""
        from .init import init_network_params
        a, c = self.actor, self.critic
        online = init_network_params(a.s_dim, a.a_dim, a.h1, a.h2, seed, c.h1, c.h2)
        target = init_network_params(a.s_dim, a.a_dim, a.h1, a.h2, seed + 1, c.h1, c.h2)
        self.set_params(_lib.ACTOR, online[0])
        self.set_params(_lib.CRITIC, online[1])
        self.set_params(_lib.ACTOR_TARGET, target[0])
        self.set_params(_lib.CRITIC_TARGET, target[1])

    def close(self):
        if self.ctx:
            lib.ddpg_destroy(self.ctx)
            self.ctx = _lib.ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- flat parameter I/O (checkpoint order)
    def param_count(self, which):
        n = _lib.ctypes.c_size_t()
        check(lib.ddpg_param_count(self.ctx, which, _lib.ctypes.byref(n)), self.ctx)
        return n.value

    def set_params(self, which, tensors):
        flat = np.concatenate([f32(t).ravel() for t in tensors]) if isinstance(
            tensors, (list, tuple)) else f32(tensors).ravel()
        check(lib.ddpg_set_params(self.ctx, which, fptr(flat), flat.size), self.ctx)

    def get_params(self, which, split=True):
        n = self.param_count(which)
        out = np.empty(n, np.float32)
        check(lib.ddpg_get_params(self.ctx, which, fptr(out), n), self.ctx)
        if not split:
            return out
        shapes = self.actor.shapes() if which in (0, 1, 4, 5, 8) else self.critic.shapes()
        res, o = [], 0
        for s in shapes:
            k = int(np.prod(s))
            res.append(out[o:o + k].reshape(s))
            o += k
        return res

    def set_adam_powers(self, net, b1p, b2p):
        check(lib.ddpg_set_adam_powers(self.ctx, net, b1p, b2p), self.ctx)

    def get_adam_powers(self, net):
        a, b = _lib.ctypes.c_float(), _lib.ctypes.c_float()
        check(lib.ddpg_get_adam_powers(self.ctx, net, _lib.ctypes.byref(a),
                                       _lib.ctypes.byref(b)), self.ctx)
        return a.value, b.value

    def sync(self):
        check(lib.ddpg_sync(self.ctx), self.ctx)

    def _rows(self, x, cols, any_batch=False):
        """[B, cols] fp32 rows.  Training calls (batch statistics) need
        1 <= B <= batch_max; forward-only calls (any_batch) take any B, as a
        TF feed does -- their rows are independent, so a batch past
        batch_max runs in batch_max-row pieces and B = 0 returns empty."""
        a = f32(x)
        if a.ndim == 1:
            a = a.reshape(-1, cols)
        if a.ndim != 2 or a.shape[1] != cols:
            raise ValueError("expected [B, %d] input, got %s" % (cols, a.shape))
        if not any_batch and (a.shape[0] > self.batch_max or a.shape[0] == 0):
            raise ValueError("batch %d outside [1, %d]" % (a.shape[0], self.batch_max))
        return a

    def _pieces(self, B):
        return [(i, min(B, i + self.batch_max)) for i in range(0, B, self.batch_max)]

    def _rowwise(self, fn, ins, width):
        """[B, width] fp32 result of fn(inputs, n, out) over row pieces of at
        most batch_max rows (one direct call when B fits: action selection
        pays no extra copy)."""
        B = ins[0].shape[0]
        out = np.empty((B, width), np.float32)
        if 0 < B <= self.batch_max:
            fn(ins, B, out)
            return out
        for i, j in self._pieces(B):
            op = np.empty((j - i, width), np.float32)
            fn([np.ascontiguousarray(x[i:j]) for x in ins], j - i, op)
            out[i:j] = op
        return out


_IO_FLOATS = 4096  # staging floats for small forward calls (Session._io_*)


def _transform(scaler, x):
    # without a scaler the rows go straight to the fp32 feed cast, as the
    # reference's preprocess_input returns them unchanged (networks.py:65-69)
    return scaler.transform(np.asarray(x, dtype=np.float64)) if scaler is not None else x


class ActorNetwork:
    """networks.py:8-99.  Input: state; output: scale * tanh(...) action."""

    def __init__(self, state_dim, action_dim, action_scale, learning_rate, tau, scaler,
                 h1=128, h2=200, graph=None):
        self.s_dim = state_dim
        self.a_dim = action_dim
        self.learning_rate = learning_rate
        self.tau = tau
        self.scaler = scaler
        self.action_scale = action_scale
        self.h1, self.h2 = h1, h2
        self.sess = None
        self.num_trainable_vars = 10  # 5 online + 5 target variables (networks.py:49)
        (graph or _default_graph).actor = self

    def shapes(self):
        S, A, H1, H2 = self.s_dim, self.a_dim, self.h1, self.h2
        return [(S, H1), (H1,), (H1, H2), (H2,), (H2, A)]

    def preprocess_input(self, inputs):
        return _transform(self.scaler, inputs)

    def train(self, inputs, a_gradient):
        ss = self.sess
        s = ss._rows(self.preprocess_input(inputs), self.s_dim)
        g = f32(a_gradient).reshape(s.shape[0], self.a_dim)
        check(lib.ddpg_actor_train(ss.ctx, fptr(s), fptr(g), s.shape[0]), ss.ctx)

    def _forward(self, inputs, target):
        ss = self.sess
        s = ss._rows(self.preprocess_input(inputs), self.s_dim, any_batch=True)
        B, S, A = s.shape[0], self.s_dim, self.a_dim
        if 0 < B <= ss.batch_max and B * max(S, A) <= _IO_FLOATS:
            # action selection (ddpg.py:68-70): staged through the session's
            # ctypes arrays
            ss._io_in_np[:B * S] = s.reshape(-1)
            check(lib.ddpg_actor_forward(ss.ctx, int(target), ss._io_in, B, ss._io_out), ss.ctx)
            return ss._io_out_np[:B * A].reshape(B, A).copy()
        fn = lambda x, n, o: check(lib.ddpg_actor_forward(ss.ctx, int(target), fptr(x[0]), n,
                                                          fptr(o)), ss.ctx)
        return ss._rowwise(fn, [s], A)

    def predict(self, inputs):
        return self._forward(inputs, False)

    def predict_target(self, inputs):
        return self._forward(inputs, True)

    def update_target_network(self):
        check(lib.ddpg_soft_update(self.sess.ctx, _lib.SOFT_ACTOR), self.sess.ctx)

    def get_num_trainable_vars(self):
        return self.num_trainable_vars

    def restore_params(self, parameters):
        """networks.py:93-96: parameters[0:5] online, parameters[5:10] target."""
        n = len(self.shapes())
        self.sess.set_params(_lib.ACTOR, [np.asarray(p) for p in parameters[:n]])
        self.sess.set_params(_lib.ACTOR_TARGET, [np.asarray(p) for p in parameters[n:2 * n]])

    def set_session(self, sess):
        self.sess = sess


class CriticNetwork:
    """networks.py:102-207.  Input: (state, action); output: Q(s, a)."""

    def __init__(self, state_dim, action_dim, learning_rate, tau, num_actor_vars, scaler,
                 h1=128, h2=200, graph=None):
        self.s_dim = state_dim
        self.a_dim = action_dim
        self.learning_rate = learning_rate
        self.tau = tau
        self.num_actor_vars = num_actor_vars
        self.scaler = scaler
        self.h1, self.h2 = h1, h2
        self.sess = None
        self.num_trainable_vars = 16  # 8 online + 8 target variables (networks.py:145)
        (graph or _default_graph).critic = self

    def shapes(self):
        S, A, H1, H2 = self.s_dim, self.a_dim, self.h1, self.h2
        return [(S, H1), (H1,), (A, H1), (H1,), (2 * H1, H2), (H2,), (H2, 1), (1,)]

    def preprocess_input(self, inputs):
        return _transform(self.scaler, inputs)

    def train(self, inputs, action, predicted_q_value):
        """Returns [out (pre-update Q, [B,1] f32), None (optimize), loss (f32)]."""
        ss = self.sess
        s = ss._rows(self.preprocess_input(inputs), self.s_dim)
        B = s.shape[0]
        a = f32(action).reshape(B, self.a_dim)
        y = f32(predicted_q_value).reshape(B, 1)
        q = np.empty((B, 1), np.float32)
        loss = _lib.ctypes.c_float()
        check(lib.ddpg_critic_train(ss.ctx, fptr(s), fptr(a), fptr(y), B, fptr(q),
                                    _lib.ctypes.byref(loss)), ss.ctx)
        return [q, None, np.float32(loss.value)]

    def _forward(self, inputs, action, target):
        ss = self.sess
        s = ss._rows(self.preprocess_input(inputs), self.s_dim, any_batch=True)
        a = f32(action).reshape(s.shape[0], self.a_dim)
        fn = lambda x, n, o: check(lib.ddpg_critic_forward(ss.ctx, int(target), fptr(x[0]),
                                                           fptr(x[1]), n, fptr(o)), ss.ctx)
        return ss._rowwise(fn, [s, a], 1)

    def predict(self, inputs, action):
        return self._forward(inputs, action, False)

    def predict_target(self, inputs, action):
        return self._forward(inputs, action, True)

    def action_gradients(self, inputs, actions):
        """networks.py:189-193: list of one [B, A] array (grad_ys = 1)."""
        ss = self.sess
        s = ss._rows(self.preprocess_input(inputs), self.s_dim, any_batch=True)
        a = f32(actions).reshape(s.shape[0], self.a_dim)
        # grad_ys = 1 per row: the rows are independent
        fn = lambda x, n, o: check(lib.ddpg_critic_action_grad(ss.ctx, fptr(x[0]), fptr(x[1]), n,
                                                               fptr(o)), ss.ctx)
        return [ss._rowwise(fn, [s, a], self.a_dim)]

    def update_target_network(self):
        check(lib.ddpg_soft_update(self.sess.ctx, _lib.SOFT_CRITIC), self.sess.ctx)

    def get_num_trainable_vars(self):
        return self.num_trainable_vars

    def restore_params(self, parameters):
        """networks.py:201-204: parameters[num_actor_vars + 0:8] online, +8:16 target."""
        n, k = len(self.shapes()), self.num_actor_vars
        self.sess.set_params(_lib.CRITIC, [np.asarray(p) for p in parameters[k:k + n]])
        self.sess.set_params(_lib.CRITIC_TARGET,
                             [np.asarray(p) for p in parameters[k + n:k + 2 * n]])

    def set_session(self, sess):
        self.sess = sess
