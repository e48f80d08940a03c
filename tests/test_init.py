"""Initialiser statistics against the reference graph's
own initializer constants (tests/golden/meta_constants.json, read from
InvertedPendulum/model_ddpg/model-1410.meta): tflearn's truncated normal
(stddev 0.02, re-drawn beyond 2 sigma) for the hidden weights, U(-0.003,
0.003) for the output layers, zero biases (networks.py:54-59,151-161), and
independent draws for the target networks (ddpg.py:224-229 then blends them
once).  TF's Philox stream is not reproducible outside TF, so the values are
not bitwise the reference's: the test pins the distributions."""
import json
import os

import numpy as np
import pytest

from distributed_ddpg_amd.init import init_network_params

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _consts():
    return json.load(open(os.path.join(GOLD, "meta_constants.json")))["consts"]


def test_initializer_constants_in_the_reference_graph():
    k = _consts()
    std = {v for n, v in k.items() if n.endswith("truncated_normal/stddev")}
    umax = {v for n, v in k.items() if n.endswith("random_uniform/max")}
    umin = {v for n, v in k.items() if n.endswith("random_uniform/min")}
    assert std == {float(np.float32(0.02))}
    assert umax == {float(np.float32(0.003))} and umin == {float(np.float32(-0.003))}
    # 2 graphs' worth of layers: actor 3 + critic 4 FullyConnected layers per
    # network copy (online, target): 5 hidden + 2 output initialisers each
    assert sum(n.endswith("truncated_normal/stddev") for n in k) == 10
    assert sum(n.endswith("random_uniform/max") for n in k) == 4


@pytest.mark.parametrize("S,A,H1,H2", [(4, 1, 128, 200), (64, 16, 1024, 1024)])
def test_initializer_statistics(S, A, H1, H2):
    k = _consts()
    std = next(v for n, v in k.items() if n.endswith("truncated_normal/stddev"))
    umax = next(v for n, v in k.items() if n.endswith("random_uniform/max"))
    actor, critic = init_network_params(S, A, H1, H2, seed=7)
    W1, b1, W2, b2, W3 = actor
    Ws, bs, Wa, ba, Wh, bh, Wo, bo = critic
    shapes = [(S, H1), (H1,), (H1, H2), (H2,), (H2, A)]
    assert [w.shape for w in actor] == shapes
    assert [w.shape for w in critic] == [(S, H1), (H1,), (A, H1), (H1,), (2 * H1, H2), (H2,),
                                         (H2, 1), (1,)]
    assert all(w.dtype == np.float32 for w in actor + critic)
    for b in (b1, b2, bs, ba, bh, bo):
        assert not b.any()
    hidden = np.concatenate([w.ravel() for w in (W1, W2, Ws, Wa, Wh)]).astype(np.float64)
    # truncated at 2 sigma: every value inside, the tails reached
    assert np.abs(hidden).max() <= 2 * std * (1 + 1e-6)
    assert np.abs(hidden).max() > 1.9 * std
    # N(0, s) truncated at +-2s: variance s^2 (1 - 2*2*phi(2) / (2 Phi(2) - 1))
    phi2 = np.exp(-2.0) / np.sqrt(2 * np.pi)
    Z = 0.9544997361036416  # 2 Phi(2) - 1
    sd_trunc = std * np.sqrt(1 - 4 * phi2 / Z)
    n = hidden.size
    assert abs(hidden.mean()) < 5 * sd_trunc / np.sqrt(n)
    assert abs(hidden.std() / sd_trunc - 1) < 5 * np.sqrt(0.5 / n) + 1e-3
    out = np.concatenate([W3.ravel(), Wo.ravel()]).astype(np.float64)
    assert out.min() >= -umax and out.max() <= umax
    if out.size >= 1000:  # U(-a, a): std a / sqrt(3)
        assert abs(out.std() / (umax / np.sqrt(3)) - 1) < 0.1


def test_target_networks_drawn_independently():
    # networks.Session draws the targets with seed + 1 (ddpg.py:224-229: own
    # random init, then one tau-blend toward the online networks)
    a0, c0 = init_network_params(4, 1, 128, 200, seed=11)
    a1, c1 = init_network_params(4, 1, 128, 200, seed=12)
    for x, y in zip(a0 + c0, a1 + c1):
        if x.any():
            assert not np.array_equal(x, y)
            r = np.corrcoef(x.ravel(), y.ravel())[0, 1]
            assert abs(r) < 0.2
    # deterministic per seed
    a2, c2 = init_network_params(4, 1, 128, 200, seed=11)
    assert all(np.array_equal(x, y) for x, y in zip(a0 + c0, a2 + c2))
