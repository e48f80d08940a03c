"""ReplayBuffer with the reference interface (replay_buffer.py:10-51), backed by
a device-resident ring buffer and a host MT19937 sampler that reproduces
CPython's random.seed / random.sample bit for bit.

Differences from the reference, by design:
  * the sampler state is owned by the buffer instead of the process-global
    `random` module (the reference seeds the global RNG at replay_buffer.py:19;
    nothing else in the learner path draws from it, so the index stream is
    identical);
  * the ring's precision follows the first rows added, as the reference's
    deque keeps whatever it is given: float64 states (what gym envs emit) give
    a float64 ring (s, s2, r kept exactly; sample_batch returns the stored
    values and the fused step applies the scaler to the unrounded state, then
    rounds once, like preprocess_input + feed_dict); float32 rows give a
    float32 ring (half the HBM; the bench's synthetic rows).  sample_batch
    returns s, r, s2 as float64 and t as bool, like np.array stacking of the
    reference's tuples;
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
        self._rb = None  # created on first add, when the row dims and precision are known
        self._one = None  # single-row staging (set up after the first add)
        self.s_dim = self.a_dim = None
        self.f64 = False

    # -- internals
    def _ensure(self, s_dim, a_dim, f64):
        if self._rb is None:
            self._rb = ctypes.c_void_p()
            check(lib.ddpg_replay_create_ex(self.device, s_dim, a_dim, self.buffer_size,
                                            self.random_seed, _lib.REPLAY_F64 if f64 else 0,
                                            ctypes.byref(self._rb)))
            self.s_dim, self.a_dim = s_dim, a_dim
            self.f64 = bool(f64)
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
        """replay_buffer.py:21-28 (one transition)."""
        w = self._one
        if w is None:
            s = np.asarray(s)
            f64 = s.dtype == np.float64 if self._rb is None else self.f64
            dt = np.float64 if f64 else np.float32
            self.add_batch(np.asarray(s, dt).reshape(1, -1),
                           np.asarray(a, np.float32).reshape(1, -1), np.array([r], dt),
                           np.array([bool(t)]), np.asarray(s2, dt).reshape(1, -1))
            self._one_setup()
            return
        # a worker's per-env-step add: through persistent ctypes arrays
        # (numpy's .ctypes pointer conversion costs microseconds per array)
        if np.size(s) != self.s_dim or np.size(s2) != self.s_dim or np.size(a) != self.a_dim:
            raise ValueError("row dims changed: expected s/s2 of %d and a of %d values" % (
                self.s_dim, self.a_dim))
        w["s_np"][:] = np.ravel(s)
        w["s2_np"][:] = np.ravel(s2)
        w["a_np"][:] = np.ravel(a)
        if not np.isscalar(r):  # a one-element array or list (some envs' rewards)
            rr = np.ravel(r)
            if rr.size != 1:
                raise ValueError("reward must be a scalar, got %d values" % rr.size)
            r = rr[0]
        w["r_np"][0] = r
        w["t"][0] = 1 if t else 0
        self._err(w["fn"](self._rb, w["s"], w["a"], w["r"], w["t"], w["s2"], 1))
        self.count = min(self.count + 1, self.buffer_size)

    def _one_setup(self):
        ct = ctypes.c_double if self.f64 else ctypes.c_float
        w = {"s": (ct * self.s_dim)(), "s2": (ct * self.s_dim)(), "r": (ct * 1)(),
             "a": (ctypes.c_float * self.a_dim)(), "t": (ctypes.c_uint8 * 1)(),
             "fn": lib.ddpg_replay_add_f64 if self.f64 else lib.ddpg_replay_add}
        for k in ("s", "s2", "r", "a"):
            w[k + "_np"] = np.ctypeslib.as_array(w[k])
        self._one = w

    def add_batch(self, s, a, r, t, s2):
        """n transitions at once (rows of s, a, r, t, s2)."""
        s = np.asarray(s)
        f64 = s.dtype == np.float64 if self._rb is None else self.f64
        dt = np.float64 if f64 else np.float32
        s = np.ascontiguousarray(s, dt)
        s2 = np.ascontiguousarray(s2, dt)
        a = np.ascontiguousarray(a, np.float32)
        n = s.shape[0]
        r = np.ascontiguousarray(np.asarray(r, dt).reshape(n))
        t = np.ascontiguousarray(np.asarray(t).reshape(n).astype(np.uint8))
        self._ensure(s.shape[1], a.shape[1], f64)
        u8 = t.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        if f64:
            rc = lib.ddpg_replay_add_f64(self._rb, _lib.dptr(s), _lib.fptr(a), _lib.dptr(r), u8,
                                         _lib.dptr(s2), n)
        else:
            rc = lib.ddpg_replay_add(self._rb, _lib.fptr(s), _lib.fptr(a), _lib.fptr(r), u8,
                                     _lib.fptr(s2), n)
        self._err(rc)
        self.count = int(lib.ddpg_replay_size(self._rb))

    def size(self):
        return self.count

    def sample_batch(self, batch_size, return_indices=False):
        if self._rb is None:
            empty = np.zeros((0,))
            return (empty, empty, empty, empty.astype(bool), empty)
        k = min(int(batch_size), self.count)
        S, A = self.s_dim, self.a_dim
        n = max(k, 1)
        s, s2, r = np.empty((n, S)), np.empty((n, S)), np.empty(n)
        a = np.empty((n, A), np.float32)
        t = np.empty(n, np.uint8)
        idx = np.empty(n, np.int64)
        got = self._err(lib.ddpg_replay_sample_batch_f64(
            self._rb, int(batch_size), _lib.dptr(s), _lib.fptr(a), _lib.dptr(r),
            t.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), _lib.dptr(s2),
            idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
        out = (s[:got], a[:got], r[:got], t[:got].astype(bool), s2[:got])
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
