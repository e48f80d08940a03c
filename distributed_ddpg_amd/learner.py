"""Fused learner step (ddpg.py:86-113 as ONE device call) and the
synchronous data-parallel plumbing that replaces the TF parameter server.

`FusedLearner.step()` = ddpg_learner_step: host MT19937 draw of the global
batch (identical on every rank) -> this rank's slice gathered from the device
ring -> target fwd + TD target -> critic train (RCCL sum of critic grads) ->
actor fwd + dQ/da -> actor train (RCCL sum of actor grads) -> soft updates.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, lib


def rccl_unique_id():
    buf = ctypes.create_string_buffer(128)
    check(lib.ddpg_comm_unique_id(buf))
    return buf.raw


def init_comm(sess, rank, world, pg=None, single=False):
    """Create the RCCL communicator of this rank's context.  The 128-byte
    unique id is broadcast from rank 0 over torch.distributed (any backend;
    gloo in CPU tests).  This is the replacement of the reference's
    tf.train.ClusterSpec/Server rendezvous (ddpg.py:168-174).

    world == 1 creates no communicator unless `single` is set: then a 1-rank
    RCCL communicator runs the data-parallel exchange as an identity through
    the same call sites as world > 1 (a one-GPU test of them)."""
    if world <= 1:
        if single:
            check(lib.ddpg_comm_init(sess.ctx, rccl_unique_id(), 1, 0), sess.ctx)
        return
    import torch.distributed as dist
    obj = [rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=pg)
    check(lib.ddpg_comm_init(sess.ctx, obj[0], world, rank), sess.ctx)


class FusedLearner:
    def __init__(self, sess, replay, batch_size):
        self.sess = sess
        self.replay = replay
        self.batch_size = int(batch_size)
        self._stats = _lib.Stats()
        a = sess.actor
        if a.scaler is not None and hasattr(a.scaler, "mean_"):
            mean = np.ascontiguousarray(a.scaler.mean_, np.float64)
            scale = np.ascontiguousarray(a.scaler.scale_, np.float64)
            check(lib.ddpg_set_scaler(sess.ctx, mean.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                      scale.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                      mean.size), sess.ctx)

    def step(self, stats=False):
        st = ctypes.byref(self._stats) if stats else None
        check(lib.ddpg_learner_step(self.sess.ctx, self.replay.handle, self.batch_size, st),
              self.sess.ctx)
        if stats:
            return self._stats.q_max, self._stats.loss
        return None

    def step_indices(self, idx, stats=False):
        idx = np.ascontiguousarray(idx, np.int64)
        st = ctypes.byref(self._stats) if stats else None
        check(lib.ddpg_learner_step_indices(
            self.sess.ctx, self.replay.handle, idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
            idx.size, st), self.sess.ctx)
        if stats:
            return self._stats.q_max, self._stats.loss
        return None

    def step_counts(self):
        """(graph-replayed steps, eager steps, capture_failed) of this context
        so far (ddpg_step_counts)."""
        return step_counts(self.sess)

    def read_stats(self, reset=True):
        q, l, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
        check(lib.ddpg_read_stats(self.sess.ctx, ctypes.byref(q), ctypes.byref(l),
                                  ctypes.byref(n), int(reset)), self.sess.ctx)
        return q.value, l.value, n.value


def step_counts(sess):
    g, e, f = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int()
    check(lib.ddpg_step_counts(sess.ctx, ctypes.byref(g), ctypes.byref(e), ctypes.byref(f)),
          sess.ctx)
    return g.value, e.value, bool(f.value)


def fill_synthetic(replay, s_dim, a_dim, n, scale=1.0, seed=0, chunk=65536):
    """SURVEY.md §8(d) synthetic transitions: s, s2 ~ N(0,1); a ~ U(-1,1)*scale;
    r ~ N(0,1); done ~ Bernoulli(0.01).  Seeded numpy PCG64."""
    rng = np.random.default_rng(seed)
    done = 0
    while done < n:
        m = min(chunk, n - done)
        s = rng.standard_normal((m, s_dim), dtype=np.float32)
        s2 = rng.standard_normal((m, s_dim), dtype=np.float32)
        a = (rng.uniform(-1, 1, (m, a_dim)) * scale).astype(np.float32)
        r = rng.standard_normal(m, dtype=np.float32)
        t = rng.random(m) < 0.01
        replay.add_batch(s, a, r, t, s2)
        done += m


class Profile:
    """Per-kernel-class HIP-event timing collected by the library."""

    def __init__(self, sess):
        self.sess = sess

    def enable(self, on=True):
        check(lib.ddpg_profile_enable(self.sess.ctx, int(on)), self.sess.ctx)

    def read(self, n=64):
        names = (ctypes.c_char * 64 * n)()
        ms = (ctypes.c_double * n)()
        la = (ctypes.c_int64 * n)()
        fl = (ctypes.c_double * n)()
        by = (ctypes.c_double * n)()
        k = check(lib.ddpg_profile_read(self.sess.ctx, n, ctypes.cast(names, ctypes.c_void_p), ms,
                                        la, fl, by), self.sess.ctx)
        out = {}
        for i in range(k):
            nm = bytes(names[i]).split(b"\0", 1)[0].decode()
            out[nm] = {"ms": ms[i], "launches": la[i], "flops": fl[i], "bytes": by[i]}
        return out
