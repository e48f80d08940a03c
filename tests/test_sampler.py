"""Replay index parity, CPU only (host sampler of libddpg_hip.so).

Bar: bit-exact.  Oracles: CPython's own `random` (the reference calls
random.seed / random.sample directly, replay_buffer.py:19,36-39) and the
golden index streams produced by importing the reference ReplayBuffer
(tests/golden/replay_indices.npz, made by tests/golden/make_fixtures.py).
"""
import json
import os
import random

import numpy as np
import pytest

from distributed_ddpg_amd.replay_buffer import Sampler

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("seed", [0, 1, 123, 1234, -5, 2 ** 32 - 1, 2 ** 32, 2 ** 40 + 5,
                                  2 ** 63 - 1])
def test_genrand_matches_cpython(seed):
    ref = random.Random(seed)
    ours = Sampler(seed).genrand(2000)  # crosses a 624-word regeneration
    exp = np.array([ref.getrandbits(32) for _ in range(2000)], np.uint32)
    assert np.array_equal(ours, exp)


def _cases():
    out = []
    for k in (1, 2, 5, 6, 7, 8, 16, 63, 64, 65, 256, 1000, 4096):
        for n in sorted({k, k + 1, 2 * k, 21 + 4 ** int(np.ceil(np.log(3 * k) / np.log(4)))
                         if k > 5 else 21, 300, 5000, 1_000_000}):
            if n >= k:
                out.append((n, k))
    return out


@pytest.mark.parametrize("n,k", _cases())
def test_sample_matches_cpython(n, k):
    for seed in (1234, 7):
        ref = random.Random(seed)
        ours = Sampler(seed)
        for _ in range(3):  # consecutive draws share the stream
            exp = ref.sample(range(n), k)
            got = ours.sample(n, k)
            assert got.tolist() == exp


def test_setsize_boundaries_exhaustive_small():
    """Every k in [0, 200] at n on both sides of the pool/set threshold."""
    ref = random.Random(99)
    ours = Sampler(99)
    for k in range(0, 201):
        setsize = 21 + (4 ** int(np.ceil(np.log(k * 3) / np.log(4))) if k > 5 else 0)
        for n in (max(k, setsize - 1), max(k, setsize), setsize + 1):
            assert ours.sample(n, k).tolist() == ref.sample(range(n), k)


def test_invalid_sample_raises():
    from distributed_ddpg_amd._lib import DDPGError
    with pytest.raises(DDPGError):
        Sampler(1).sample(3, 4)


def test_golden_replay_streams():
    """Emulate the reference deque -> positions -> insertion indices with the
    host sampler and compare to the streams produced by the reference code."""
    z = np.load(os.path.join(GOLD, "replay_indices.npz"))
    cases = json.loads(bytes(z["__cases__"]).decode())
    assert len(cases) >= 10
    for case in cases:
        smp = Sampler(case["seed"])
        cap, total, j = case["capacity"], 0, 0
        for op, n in case["ops"]:
            if op == "add":
                total += n
                continue
            count = min(total, cap)
            k = min(n, count)
            pos = smp.sample(count, k)
            ins = (total - count) + pos
            exp = z["%s__%d" % (case["name"], j)]
            assert np.array_equal(ins, exp), case["name"]
            j += 1
