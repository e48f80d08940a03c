"""Parameter initialisation with the reference's tflearn defaults.

networks.py:54-59,151-161 (constants confirmed in the .meta graphs, see
tests/golden/meta_constants.json): hidden W ~ TruncatedNormal(0, 0.02)
(re-drawn beyond 2 sigma), biases 0, output-layer W ~ U(-0.003, 0.003),
critic output bias 0.  TF's Philox streams are not reproducible outside TF,
so draws come from numpy's PCG64 with the given seed.
"""
import numpy as np


def _trunc_normal(rng, shape, std=0.02):
    x = rng.standard_normal(shape)
    bad = np.abs(x) > 2.0
    while bad.any():
        x[bad] = rng.standard_normal(int(bad.sum()))
        bad = np.abs(x) > 2.0
    return (std * x).astype(np.float32)


def init_network_params(S, A, H1, H2, seed, CH1=None, CH2=None):
    """Returns (actor_list, critic_list) in checkpoint order.  Critic widths
    default to the actor's (the committed networks.py uses 128/200 for both)."""
    CH1, CH2 = CH1 or H1, CH2 or H2
    rng = np.random.default_rng(seed)
    z = lambda *s: np.zeros(s, np.float32)
    u = lambda *s: rng.uniform(-0.003, 0.003, s).astype(np.float32)
    actor = [_trunc_normal(rng, (S, H1)), z(H1), _trunc_normal(rng, (H1, H2)), z(H2), u(H2, A)]
    critic = [_trunc_normal(rng, (S, CH1)), z(CH1), _trunc_normal(rng, (A, CH1)), z(CH1),
              _trunc_normal(rng, (2 * CH1, CH2)), z(CH2), u(CH2, 1), z(1)]
    return actor, critic
