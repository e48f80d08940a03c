"""Pin the oracle to the reference's own TF graphs.

Three fixtures, each a 3-step learner trajectory produced by EXECUTING one of
the reference's MetaGraphDefs (TF 1.3) from its own checkpoint (see
make_graph_fixtures.py / tfgraph.py):
  ip1410        InvertedPendulum graph (model-1410.meta), its checkpoint's
                weights, targets, Adam slots (t ~ 1.4e5) and beta powers (0.0:
                underflowed, so alpha = lr exactly)
  ip1410_fresh  the same graph and weights with the optimizer state the
                graph's own initializers give (slots 0, beta powers 0.9 /
                0.999): Adam bias correction (networks.py:47,137 ApplyAdam's
                beta1_power / beta2_power inputs and the Adam/Assign power
                updates) is exercised -- step 1 applies alpha = 0.316 lr
  ip1410_b256   the ip1410 start at the reference's default batch of 256
                (parameters.py:11): on the GPU it runs the large-batch GEMM path
  mc120         the MountainCar graph (results/model_ddpg/model-120.meta: S=2,
                actor 48/64, critic 48/128, the older networks.py whose actor
                output is the tanh itself) from its own checkpoint (t ~ 45k),
                fed states through a fitted StandardScaler (networks.py:65-69,
                164-168)
The oracle's restatement of networks.py / ddpg.py:86-113, started from the same
state and fed the same batches, must reproduce every intermediate (target Q,
TD target, pre-update Q, loss, a_outs, dQ/da), every gradient an ApplyAdam
consumed, and the final weights / targets / Adam slots / beta powers.  Fixture
arrays are stored as float32, so the bar is a few float32 ulps (rel 1e-6); a
wiring difference (wrong operand, missing grad_ys sign, post- vs pre-update
critic, missing bias correction) is O(1).

The kernel FORMULAS (Elu, EluGrad, TanhGrad, ApplyAdam) are restated in both
the interpreter and the oracle; this pins the graph wiring, not TF's kernels.
"""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")
TOL = 1e-6

# fixture: (file, S, A, actor H1/H2, critic H1/H2, action scale)
FIXTURES = {
    "ip1410": ("graph_ip1410.npz", 4, 1, (128, 200), (128, 200), 3.0),
    "ip1410_fresh": ("graph_ip1410_fresh.npz", 4, 1, (128, 200), (128, 200), 3.0),
    "mc120": ("graph_mc120.npz", 2, 1, (48, 64), (48, 128), 1.0),
    # the reference default batch (parameters.py:11): B = 256 rows per step
    "ip1410_b256": ("graph_ip1410_b256.npz", 4, 1, (128, 200), (128, 200), 3.0),
}


def rel(x, ref):
    x = np.asarray(x, np.float64)
    ref = np.asarray(ref, np.float64).reshape(x.shape)
    return float(np.max(np.abs(x - ref)) / max(np.max(np.abs(ref)), 1e-30))


class FixedScaler:
    """A fitted sklearn StandardScaler's transform (mean_, scale_; float64)."""

    def __init__(self, mean, scale):
        self.mean_ = np.asarray(mean, np.float64)
        self.scale_ = np.asarray(scale, np.float64)

    def transform(self, x):
        return (np.asarray(x, np.float64) - self.mean_) / self.scale_


def fixture(name):
    """(z, dims, start params, scaler or None) of a graph fixture."""
    fn, S, A, (H1, H2), (CH1, CH2), scale = FIXTURES[name]
    z = np.load(os.path.join(GOLD, fn))
    w = z if "init/FullyConnected/W" in z.files else np.load(os.path.join(GOLD,
                                                                         "ip_model1410.npz"))
    pfx = "init/" if w is z else ""
    from oracle import ddpg_oracle as O
    get = lambda names, keys: {k: w[pfx + n] for k, n in zip(keys, names)}
    p = {"actor": get(O.CKPT_ACTOR, O.ACTOR_KEYS), "actor_t": get(O.CKPT_ACTOR_T, O.ACTOR_KEYS),
         "critic": get(O.CKPT_CRITIC, O.CRITIC_KEYS),
         "critic_t": get(O.CKPT_CRITIC_T, O.CRITIC_KEYS)}
    scaler = FixedScaler(z["scaler/mean"], z["scaler/scale"]) if "scaler/mean" in z.files else None
    return z, (S, A, H1, H2, CH1, CH2, scale), p, scaler


def load_fixture_learner(O, dtype=np.float64, name="ip1410"):
    """Oracle Learner at the fixture's initial state (weights, Adam slots, powers)."""
    z, (S, A, H1, H2, CH1, CH2, scale), p, _ = fixture(name)
    L = O.Learner(S, A, H1, H2, scale, dtype=dtype, params=p, init_blend=False, CH1=CH1, CH2=CH2)
    for opt, names, keys, sfx in ((L.actor_opt, O.CKPT_ACTOR, O.ACTOR_KEYS, ""),
                                  (L.critic_opt, O.CKPT_CRITIC, O.CRITIC_KEYS, "_1")):
        for k, n in zip(keys, names):
            opt.m[k] = z["init/%s/Adam" % n].astype(dtype)
            opt.v[k] = z["init/%s/Adam_1" % n].astype(dtype)
        opt.b1p = dtype(z["init/beta1_power" + sfx])
        opt.b2p = dtype(z["init/beta2_power" + sfx])
    return L, p, z


@pytest.mark.parametrize("name", list(FIXTURES))
def test_oracle_reproduces_reference_graph_trajectory(name):
    from oracle import ddpg_oracle as O
    L, _, z = load_fixture_learner(O, name=name)
    scaler = fixture(name)[3]
    pre = (lambda x: x) if scaler is None else scaler.transform
    for step in range(3):
        p = "step%d/" % step
        out = L.step(pre(z[p + "s"]), z[p + "a"], z[p + "r"], z[p + "t"], pre(z[p + "s2"]))
        assert rel(out["y"], z[p + "y"]) < TOL, step
        assert rel(out["q"], z[p + "q"]) < TOL, step
        assert abs(out["loss"] - float(z[p + "loss"])) <= TOL * abs(float(z[p + "loss"]))
        assert rel(out["a_outs"], z[p + "a_outs"]) < TOL, step
        assert rel(out["da"], z[p + "da"]) < TOL, step
        for keys, names, g in ((O.CRITIC_KEYS, O.CKPT_CRITIC, out["critic_grads"]),
                               (O.ACTOR_KEYS, O.CKPT_ACTOR, out["actor_grads"])):
            for k, n in zip(keys, names):
                assert rel(g[k], z[p + "grad/" + n]) < TOL, (step, n)
    st = L.state()
    for net, keys, names in (("actor", O.ACTOR_KEYS, O.CKPT_ACTOR),
                             ("actor_t", O.ACTOR_KEYS, O.CKPT_ACTOR_T),
                             ("critic", O.CRITIC_KEYS, O.CKPT_CRITIC),
                             ("critic_t", O.CRITIC_KEYS, O.CKPT_CRITIC_T)):
        for k, n in zip(keys, names):
            assert rel(st[net][k], z["final/" + n]) < TOL, n
    for opt, keys, names, sfx in ((L.actor_opt, O.ACTOR_KEYS, O.CKPT_ACTOR, ""),
                                  (L.critic_opt, O.CRITIC_KEYS, O.CKPT_CRITIC, "_1")):
        for k, n in zip(keys, names):
            assert rel(opt.m[k], z["final/%s/Adam" % n]) < TOL, n
            assert rel(opt.v[k], z["final/%s/Adam_1" % n]) < TOL, n
        assert opt.b1p == pytest.approx(float(z["final/beta1_power" + sfx]), rel=1e-12)
        assert opt.b2p == pytest.approx(float(z["final/beta2_power" + sfx]), rel=1e-12)


def test_graph_fixture_detects_wiring_changes():
    """The fixture is sensitive to the quirks it pins: taking dQ/da with the
    PRE-update critic, or dropping grad_ys' sign, moves the result by far more
    than the bar."""
    from oracle import ddpg_oracle as O
    L, _, z = load_fixture_learner(O)
    s, a = z["step0/s"], z["step0/a"]
    critic_before = {k: v.copy() for k, v in L.critic.items()}
    L.step(s, a, z["step0/r"], z["step0/t"], z["step0/s2"])
    da_pre = O.critic_action_grads(critic_before, s, z["step0/a_outs"])
    assert rel(da_pre, z["step0/da"]) > 100 * TOL
    L0, _, _ = load_fixture_learner(O)
    g = O.actor_grads(L0.actor, s, -z["step0/da"], 3.0)  # sign of grad_ys flipped
    assert rel(g["W1"], z["step0/grad/FullyConnected/W"]) > 1.0


def test_fresh_fixture_pins_bias_correction():
    """Step 1 of the fresh-optimizer trajectory: the graph's beta powers start
    at 0.9 / 0.999, so ApplyAdam's alpha = lr sqrt(1 - 0.999) / (1 - 0.9) =
    0.316 lr, and with m = 0.1 g, v = 0.001 g^2 every weight with |g| >> eps
    moves by lr (in the direction -sign(g)).  An Adam without bias correction
    (alpha = lr) moves them by 3.16 lr: the fixture tells the two apart."""
    from oracle import ddpg_oracle as O
    z, _, p, _ = fixture("ip1410_fresh")
    assert float(z["init/beta1_power"]) == pytest.approx(0.9, rel=1e-7)
    assert float(z["init/beta2_power_1"]) == pytest.approx(0.999, rel=1e-7)
    assert float(z["final/beta1_power"]) == pytest.approx(0.9 ** 4, rel=1e-6)
    # critic step 1 from the graph's own gradient: dtheta = -lr sign(g)
    L, _, _ = load_fixture_learner(O, name="ip1410_fresh")
    g = z["step0/grad/FullyConnected_8/W"].astype(np.float64)
    w0 = p["critic"]["Wh"].astype(np.float64)
    L.critic_opt.apply(L.critic, {"Wh": g})
    step = L.critic["Wh"] - w0
    big = np.abs(g) > 1e-2
    lr_c = float(np.float32(1e-3))
    np.testing.assert_allclose(step[big], -lr_c * np.sign(g[big]), rtol=1e-4)
    # the same update without bias correction misses the graph's trajectory
    Lnb, _, _ = load_fixture_learner(O, name="ip1410_fresh")
    for opt in (Lnb.actor_opt, Lnb.critic_opt):
        opt.b1p = opt.b2p = 0.0  # alpha = lr
    Lnb.step(z["step0/s"], z["step0/a"], z["step0/r"], z["step0/t"], z["step0/s2"])
    La, _, _ = load_fixture_learner(O, name="ip1410_fresh")
    La.step(z["step0/s"], z["step0/a"], z["step0/r"], z["step0/t"], z["step0/s2"])
    d_ok = La.critic["Wh"] - w0
    d_nb = Lnb.critic["Wh"] - w0
    assert np.max(np.abs(d_nb)) > 2.5 * np.max(np.abs(d_ok))


def test_mc_fixture_uses_scaler_and_asymmetric_widths():
    z, (S, A, H1, H2, CH1, CH2, scale), p, scaler = fixture("mc120")
    assert (S, A, H1, H2, CH1, CH2) == (2, 1, 48, 64, 48, 128)
    assert p["actor"]["W2"].shape == (48, 64) and p["critic"]["Wh"].shape == (96, 128)
    assert scaler is not None and float(z["init/beta2_power_1"]) < 1e-19
    # raw states fed unscaled miss the graph's outputs
    from oracle import ddpg_oracle as O
    L, _, _ = load_fixture_learner(O, name="mc120")
    a_raw = L.actor_predict(z["step0/s"])
    assert rel(a_raw, z["step0/a_outs"]) > 100 * TOL
