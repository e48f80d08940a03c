"""ctypes binding of libddpg_hip.so (the C-ABI declared in include/ddpg_hip.h).

The HIP extension is the product path: if the library is missing this module
raises on import -- there is no CPU fallback.  torch is imported first so that
the process has exactly one HIP runtime (torch's bundled libamdhip64.so.7 and
librccl.so.1 satisfy the library's NEEDED entries by SONAME).
"""
import ctypes
import os

import numpy as np
import torch  # noqa: F401  (must precede the library load; see module doc)

_HERE = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(_HERE)
# DDPG_LIB_PATH: a same-box A/B build for the tools/ scripts only; it must live
# under tools/ab/ or build_variants/ (the tools' own output), never elsewhere
_ALT = os.environ.get("DDPG_LIB_PATH")
if _ALT:
    _alt = os.path.realpath(_ALT)
    if not any(_alt.startswith(os.path.join(os.path.realpath(_REPO), d) + os.sep)
               for d in ("tools", "build_variants")):
        raise ImportError("DDPG_LIB_PATH=%s: only A/B builds under tools/ or build_variants/ "
                          "may replace the product library" % _ALT)
LIB_PATH = _ALT or os.path.join(_HERE, "libddpg_hip.so")

DDPG_OK = 0
DDPG_EINVAL, DDPG_EHIP, DDPG_ENOMEM, DDPG_ESTATE, DDPG_ECOMM = -1, -2, -3, -4, -5
FP32, BF16 = 0, 1
ACTOR, ACTOR_TARGET, CRITIC, CRITIC_TARGET = 0, 1, 2, 3
ACTOR_ADAM_M, ACTOR_ADAM_V, CRITIC_ADAM_M, CRITIC_ADAM_V = 4, 5, 6, 7
ACTOR_GRAD, CRITIC_GRAD = 8, 9
REPLAY_F64 = 1
ABI_VERSION = 2
SOFT_ACTOR, SOFT_CRITIC = 1, 2


class DDPGError(RuntimeError):
    """Raised for negative status codes (TF would raise InvalidArgumentError)."""

    def __init__(self, code, msg):
        super().__init__("ddpg_hip error %d: %s" % (code, msg))
        self.code = code


class Cfg(ctypes.Structure):
    _fields_ = [("state_dim", ctypes.c_int), ("action_dim", ctypes.c_int),
                ("h1", ctypes.c_int), ("h2", ctypes.c_int), ("batch_max", ctypes.c_int),
                ("actor_lr", ctypes.c_float), ("critic_lr", ctypes.c_float),
                ("tau", ctypes.c_float), ("gamma", ctypes.c_float),
                ("action_scale", ctypes.c_float), ("beta1", ctypes.c_float),
                ("beta2", ctypes.c_float), ("epsilon", ctypes.c_float),
                ("dtype", ctypes.c_int), ("device", ctypes.c_int),
                ("rank", ctypes.c_int), ("world", ctypes.c_int),
                ("critic_h1", ctypes.c_int), ("critic_h2", ctypes.c_int)]


class Stats(ctypes.Structure):
    _fields_ = [("q_max", ctypes.c_float), ("loss", ctypes.c_float)]


if not os.path.exists(LIB_PATH):
    raise ImportError("libddpg_hip.so not built (%s); run `python -c 'import __graft_entry__ as g; "
                      "g.build()'` or `make -C distributed_ddpg_amd/csrc`" % LIB_PATH)

lib = ctypes.CDLL(LIB_PATH)

_c = ctypes
_P = ctypes.c_void_p
_fp = ctypes.POINTER(ctypes.c_float)
_dp = ctypes.POINTER(ctypes.c_double)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)

# (name, restype, argtypes) -- must match include/ddpg_hip.h
PROTOTYPES = [
    ("ddpg_abi_version", _c.c_int, []),
    ("ddpg_global_error", _c.c_char_p, []),
    ("ddpg_create", _c.c_int, [_c.POINTER(Cfg), _c.POINTER(_P)]),
    ("ddpg_destroy", None, [_P]),
    ("ddpg_last_error", _c.c_char_p, [_P]),
    ("ddpg_sync", _c.c_int, [_P]),
    ("ddpg_set_stream", _c.c_int, [_P, _P]),
    ("ddpg_param_count", _c.c_int, [_P, _c.c_int, _c.POINTER(_c.c_size_t)]),
    ("ddpg_set_params", _c.c_int, [_P, _c.c_int, _fp, _c.c_size_t]),
    ("ddpg_get_params", _c.c_int, [_P, _c.c_int, _fp, _c.c_size_t]),
    ("ddpg_set_adam_powers", _c.c_int, [_P, _c.c_int, _c.c_float, _c.c_float]),
    ("ddpg_get_adam_powers", _c.c_int, [_P, _c.c_int, _fp, _fp]),
    ("ddpg_actor_forward", _c.c_int, [_P, _c.c_int, _fp, _c.c_int, _fp]),
    ("ddpg_critic_forward", _c.c_int, [_P, _c.c_int, _fp, _fp, _c.c_int, _fp]),
    ("ddpg_critic_train", _c.c_int, [_P, _fp, _fp, _fp, _c.c_int, _fp, _fp]),
    ("ddpg_critic_action_grad", _c.c_int, [_P, _fp, _fp, _c.c_int, _fp]),
    ("ddpg_actor_train", _c.c_int, [_P, _fp, _fp, _c.c_int]),
    ("ddpg_soft_update", _c.c_int, [_P, _c.c_int]),
    ("ddpg_set_scaler", _c.c_int, [_P, _dp, _dp, _c.c_int]),
    ("ddpg_sampler_create", _c.c_int, [_c.c_int64, _c.POINTER(_P)]),
    ("ddpg_sampler_destroy", None, [_P]),
    ("ddpg_sampler_sample", _c.c_int, [_P, _c.c_int64, _c.c_int, _i64p]),
    ("ddpg_sampler_getrandbits32", _c.c_int, [_P, _u32p, _c.c_int]),
    ("ddpg_replay_create", _c.c_int, [_c.c_int, _c.c_int, _c.c_int, _c.c_int64, _c.c_int64,
                                      _c.POINTER(_P)]),
    ("ddpg_replay_create_ex", _c.c_int, [_c.c_int, _c.c_int, _c.c_int, _c.c_int64, _c.c_int64,
                                         _c.c_int, _c.POINTER(_P)]),
    ("ddpg_replay_is_f64", _c.c_int, [_P]),
    ("ddpg_replay_destroy", None, [_P]),
    ("ddpg_replay_last_error", _c.c_char_p, [_P]),
    ("ddpg_replay_add", _c.c_int, [_P, _fp, _fp, _fp, _u8p, _fp, _c.c_int]),
    ("ddpg_replay_add_f64", _c.c_int, [_P, _dp, _fp, _dp, _u8p, _dp, _c.c_int]),
    ("ddpg_replay_size", _c.c_int64, [_P]),
    ("ddpg_replay_total_added", _c.c_int64, [_P]),
    ("ddpg_replay_clear", _c.c_int, [_P]),
    ("ddpg_replay_sample_batch", _c.c_int, [_P, _c.c_int, _fp, _fp, _fp, _u8p, _fp, _i64p]),
    ("ddpg_replay_sample_batch_f64", _c.c_int, [_P, _c.c_int, _dp, _fp, _dp, _u8p, _dp, _i64p]),
    ("ddpg_learner_step", _c.c_int, [_P, _P, _c.c_int, _c.POINTER(Stats)]),
    ("ddpg_learner_step_indices", _c.c_int, [_P, _P, _i64p, _c.c_int, _c.POINTER(Stats)]),
    ("ddpg_read_stats", _c.c_int, [_P, _dp, _dp, _i64p, _c.c_int]),
    ("ddpg_comm_unique_id", _c.c_int, [_c.c_char_p]),
    ("ddpg_comm_init", _c.c_int, [_P, _c.c_char_p, _c.c_int, _c.c_int]),
    ("ddpg_comm_init_proxy", _c.c_int, [_P]),
    ("ddpg_step_counts", _c.c_int, [_P, _i64p, _i64p, _c.POINTER(_c.c_int)]),
    ("ddpg_profile_enable", _c.c_int, [_P, _c.c_int]),
    ("ddpg_profile_read", _c.c_int, [_P, _c.c_int, _P, _dp, _i64p, _dp, _dp]),
    ("ddpg_crc32c", _c.c_uint32, [_c.c_uint32, _c.c_void_p, _c.c_size_t]),
]

_skipped = []
for _name, _res, _args in PROTOTYPES:
    try:
        _f = getattr(lib, _name)  # AttributeError here == ABI drift
    except AttributeError:
        # an older A/B build (DDPG_LIB_PATH) may predate entry points added
        # since: tolerated only on explicit opt-in, and named
        if _ALT and os.environ.get("DDPG_LIB_ALLOW_MISSING") == "1":
            _skipped.append(_name)
            continue
        raise
    _f.restype = _res
    _f.argtypes = _args
if _skipped:
    import warnings
    warnings.warn("%s lacks %s (DDPG_LIB_ALLOW_MISSING=1)" % (LIB_PATH, ", ".join(_skipped)))

if lib.ddpg_abi_version() != ABI_VERSION:
    raise ImportError("libddpg_hip.so ABI version mismatch")


def check(rc, ctx=None):
    if rc < 0:
        msg = lib.ddpg_last_error(ctx) if ctx else lib.ddpg_global_error()
        raise DDPGError(rc, (msg or b"").decode(errors="replace"))
    return rc


def fptr(a):
    return a.ctypes.data_as(_fp)


def dptr(a):
    return a.ctypes.data_as(_dp)


def f32(x, shape=None):
    """C-contiguous float32 copy/view (TF feed_dict cast)."""
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float32))
    if shape is not None:
        a = a.reshape(shape)
    return a
