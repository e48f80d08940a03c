"""ReplayBuffer with the reference interface (replay_buffer.py:10-51), backed by
a device-resident ring buffer and a host MT19937 sampler that reproduces
CPython's random.seed / random.sample bit for bit.

Differences from the reference, by design:
  * the sampler state is owned by the buffer instead of the process-global
    `random` module (the reference seeds the global RNG at replay_buffer.py:19;
    nothing else in the learner path draws from it, so the index stream is
    identical);
  * rows are stored in fp32 -- the precision at which the reference's
    networks consume them (TF feed_dict casts); sample_batch returns s, r, s2
    as float64 views of those values and t as bool, like np.array stacking of
    the reference's tuples;
  * clear() works (the reference's references a non-existent self.deque).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, lib


class ReplayBuffer:
    def __init__(self, buffer_size, random_seed=123, device=0):
        self.buffer_size = int(buffer_size)
        self.random_seed = int(random_seed)
        self.device = int(device)
        self.count = 0
        self._rb = None  # created on first add, when the row dims are known
        self.s_dim = self.a_dim = None

    # -- internals
    def _ensure(self, s_dim, a_dim):
        if self._rb is None:
            self._rb = ctypes.c_void_p()
            check(lib.ddpg_replay_create(self.device, s_dim, a_dim, self.buffer_size,
                                         self.random_seed, ctypes.byref(self._rb)))
            self.s_dim, self.a_dim = s_dim, a_dim
        elif (s_dim, a_dim) != (self.s_dim, self.a_dim):
            raise ValueError("row dims changed: (%d,%d) -> (%d,%d)" % (
                self.s_dim, self.a_dim, s_dim, a_dim))

    def _err(self, rc):
        if rc < 0:
            msg = lib.ddpg_replay_last_error(self._rb) if self._rb else lib.ddpg_global_error()
            raise _lib.DDPGError(rc, (msg or b"").decode())
        return rc

    @property
    def handle(self):
        return self._rb

    # -- reference interface
    def add(self, s, a, r, t, s2):
        s = np.asarray(s, np.float32).reshape(1, -1)
        a = np.asarray(a, np.float32).reshape(1, -1)
        self.add_batch(s, a, np.array([r], np.float32), np.array([bool(t)]),
                       np.asarray(s2, np.float32).reshape(1, -1))

    def add_batch(self, s, a, r, t, s2):
        s = np.ascontiguousarray(s, np.float32)
        a = np.ascontiguousarray(a, np.float32)
        s2 = np.ascontiguousarray(s2, np.float32)
        n = s.shape[0]
        r = np.ascontiguousarray(np.asarray(r, np.float32).reshape(n))
        t = np.ascontiguousarray(np.asarray(t).reshape(n).astype(np.uint8))
        self._ensure(s.shape[1], a.shape[1])
        self._err(lib.ddpg_replay_add(self._rb, _lib.fptr(s), _lib.fptr(a), _lib.fptr(r),
                                      t.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                      _lib.fptr(s2), n))
        self.count = int(lib.ddpg_replay_size(self._rb))

    def size(self):
        return self.count

    def sample_batch(self, batch_size, return_indices=False):
        if self._rb is None:
            empty = np.zeros((0,))
            return (empty, empty, empty, empty.astype(bool), empty)
        k = min(int(batch_size), self.count)
        S, A = self.s_dim, self.a_dim
        s = np.empty((max(k, 1), S), np.float32)
        s2 = np.empty((max(k, 1), S), np.float32)
        a = np.empty((max(k, 1), A), np.float32)
        r = np.empty(max(k, 1), np.float32)
        t = np.empty(max(k, 1), np.uint8)
        idx = np.empty(max(k, 1), np.int64)
        got = self._err(lib.ddpg_replay_sample_batch(
            self._rb, int(batch_size), _lib.fptr(s), _lib.fptr(a), _lib.fptr(r),
            t.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), _lib.fptr(s2),
            idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
        out = (s[:got].astype(np.float64), a[:got], r[:got].astype(np.float64),
               t[:got].astype(bool), s2[:got].astype(np.float64))
        if return_indices:
            return out + (idx[:got],)
        return out

    def clear(self):
        if self._rb is not None:
            check(lib.ddpg_replay_clear(self._rb))
        self.count = 0

    def __del__(self):
        try:
            if self._rb:
                lib.ddpg_replay_destroy(self._rb)
                self._rb = None
        except Exception:
            pass


class Sampler:
    """Host-only random.sample(range(n), k) restatement (no GPU needed)."""

    def __init__(self, seed):
        self._h = ctypes.c_void_p()
        check(lib.ddpg_sampler_create(int(seed), ctypes.byref(self._h)))

    def sample(self, n, k):
        out = np.empty(max(k, 1), np.int64)
        check(lib.ddpg_sampler_sample(self._h, int(n), int(k),
                                      out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
        return out[:k]

    def genrand(self, n):
        out = np.empty(n, np.uint32)
        check(lib.ddpg_sampler_getrandbits32(self._h, out.ctypes.data_as(
            ctypes.POINTER(ctypes.c_uint32)), n))
        return out

    def __del__(self):
        try:
            lib.ddpg_sampler_destroy(self._h)
        except Exception:
            pass
