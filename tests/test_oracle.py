"""Pin the CPU oracle (oracle/ddpg_oracle.py) before trusting it:
  * against an independent torch-fp64 autograd formulation of the reference
    graph (networks.py:51-63,147-162 + tf.gradients semantics);
  * against central finite differences for dQ/da and the actor gradient;
  * TF ApplyAdam / soft-update / TD-target arithmetic on hand-checked values;
  * against the reference's own artefacts: decoded checkpoints (shapes, the
    Adam slot / beta-power relations) and the graph constants of the .meta.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import ddpg_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _rand_params(S, A, H1, H2, seed, scale=0.3):
    rng = np.random.default_rng(seed)
    a = {k: rng.standard_normal(s) * scale for k, s in O.actor_shapes(S, A, H1, H2).items()}
    c = {k: rng.standard_normal(s) * scale for k, s in O.critic_shapes(S, A, H1, H2).items()}
    return a, c


def _torch_graph(a, c, s, act, scale):
    """Independent formulation with torch autograd (fp64)."""
    T = lambda x: torch.tensor(x, dtype=torch.float64, requires_grad=True)
    ta = {k: T(v) for k, v in a.items()}
    tc = {k: T(v) for k, v in c.items()}
    ts = torch.tensor(s, dtype=torch.float64)
    tact = T(act)
    elu = torch.nn.functional.elu
    mu = torch.tanh(elu(elu(ts @ ta["W1"] + ta["b1"]) @ ta["W2"] + ta["b2"]) @ ta["W3"]) * scale
    h = elu(torch.cat([elu(ts @ tc["Ws"] + tc["bs"]), elu(tact @ tc["Wa"] + tc["ba"])], 1)
            @ tc["Wh"] + tc["bh"])
    q = h @ tc["Wo"] + tc["bo"]
    return ta, tc, tact, mu, q


@pytest.mark.parametrize("S,A,H1,H2,B", [(4, 1, 16, 24, 9), (3, 2, 8, 12, 5), (6, 3, 20, 10, 17)])
def test_oracle_vs_torch_autograd(S, A, H1, H2, B):
    a, c = _rand_params(S, A, H1, H2, seed=S * 100 + A)
    rng = np.random.default_rng(7)
    s = rng.standard_normal((B, S))
    act = rng.standard_normal((B, A))
    y = rng.standard_normal((B, 1))
    scale = 2.5
    ta, tc, tact, mu, q = _torch_graph(a, c, s, act, scale)
    # forwards
    np.testing.assert_allclose(O.actor_forward(a, s, scale)[3], mu.detach().numpy(), rtol=1e-12)
    np.testing.assert_allclose(O.critic_forward(c, s, act)[3], q.detach().numpy(), rtol=1e-12)
    # critic loss grads (tflearn.mean_square)
    loss = torch.mean((torch.tensor(y) - q) ** 2)
    g_c = torch.autograd.grad(loss, list(tc.values()), retain_graph=True)
    lo, dq = O.mse_loss_and_grad(y, O.critic_forward(c, s, act)[3])
    assert abs(lo - loss.item()) < 1e-12 * max(1, abs(loss.item()))
    gc, _, _ = O.critic_grads(c, s, act, dq)
    for k, gt in zip(tc.keys(), g_c):
        np.testing.assert_allclose(gc[k], gt.numpy(), rtol=1e-10, atol=1e-13, err_msg=k)
    # dQ/da with grad_ys = 1 (networks.py:143)
    (g_a,) = torch.autograd.grad(q.sum(), [tact], retain_graph=True)
    np.testing.assert_allclose(O.critic_action_grads(c, s, act), g_a.numpy(), rtol=1e-10,
                               atol=1e-13)
    # actor gradient with grad_ys = -a_gradient (networks.py:44)
    dqa = rng.standard_normal((B, A))
    g_act = torch.autograd.grad(mu, list(ta.values()), grad_outputs=-torch.tensor(dqa))
    ga = O.actor_grads(a, s, dqa, scale)
    for k, gt in zip(ta.keys(), g_act):
        np.testing.assert_allclose(ga[k], gt.numpy(), rtol=1e-10, atol=1e-13, err_msg=k)


def test_finite_differences():
    S, A, H1, H2, B = 3, 2, 7, 5, 4
    a, c = _rand_params(S, A, H1, H2, seed=3)
    rng = np.random.default_rng(1)
    s = rng.standard_normal((B, S))
    act = rng.standard_normal((B, A))
    da = O.critic_action_grads(c, s, act)
    eps = 1e-6
    for b in range(B):
        for j in range(A):
            p, m = act.copy(), act.copy()
            p[b, j] += eps
            m[b, j] -= eps
            fd = (O.critic_forward(c, s, p)[3][b, 0] - O.critic_forward(c, s, m)[3][b, 0]) / (2 * eps)
            assert abs(fd - da[b, j]) < 1e-6
    dqa = rng.standard_normal((B, A))
    ga = O.actor_grads(a, s, dqa, 1.5)
    # d/dW of sum(-dqa * mu)
    f = lambda aa: float(np.sum(-dqa * O.actor_forward(aa, s, 1.5)[3]))
    for k in ("W1", "b2", "W3"):
        idx = tuple(0 for _ in a[k].shape)
        ap, am = {**a, k: a[k].copy()}, {**a, k: a[k].copy()}
        ap[k][idx] += eps
        am[k][idx] -= eps
        assert abs((f(ap) - f(am)) / (2 * eps) - ga[k][idx]) < 1e-6, k


def test_tf_adam_semantics():
    """ApplyAdam on scalars, checked against the TF 1.3 formula by hand."""
    opt = O.TFAdam({"w": (1,)}, lr=0.001, dtype=np.float64)
    p = {"w": np.array([0.5])}
    g = {"w": np.array([0.2])}
    opt.apply(p, g)
    m = 0.2 * 0.1
    v = 0.04 * 0.001
    alpha = 0.001 * np.sqrt(1 - 0.999) / (1 - 0.9)
    assert np.isclose(p["w"][0], 0.5 - m * alpha / (np.sqrt(v) + 1e-8), rtol=1e-15)
    assert np.isclose(opt.b1p, 0.81) and np.isclose(opt.b2p, 0.999 ** 2)
    # fp32 variant keeps fp32 throughout
    opt32 = O.TFAdam({"w": (1,)}, lr=0.001, dtype=np.float32)
    p32 = {"w": np.array([0.5], np.float32)}
    opt32.apply(p32, {"w": np.array([0.2], np.float32)})
    assert p32["w"].dtype == np.float32 and opt32.b1p.dtype == np.float32


def test_soft_update_and_td_target_fp32():
    th = {"w": np.array([1.0, -2.0, 3.5], np.float32)}
    tt = {"w": np.array([0.5, 0.25, -1.0], np.float32)}
    O.soft_update(th, tt, 0.001)
    exp = th["w"] * np.float32(0.001) + np.array([0.5, 0.25, -1.0], np.float32) * np.float32(0.999)
    assert np.array_equal(tt["w"], exp) and tt["w"].dtype == np.float32
    q2 = np.array([[1.5], [2.0], [-3.0]], np.float32)
    y = O.td_target(np.array([1.0, 2.0, 0.5]), np.array([False, True, False]), q2, 0.99)
    assert y.dtype == np.float32
    assert y[1, 0] == np.float32(2.0)
    assert y[0, 0] == np.float32(1.0) + np.float32(0.99) * np.float32(1.5)


def test_meta_constants_match_oracle_defaults():
    meta = json.load(open(os.path.join(GOLD, "meta_constants.json")))
    assert meta["tf_version"] == "1.3.0"
    k = meta["consts"]
    f32 = lambda x: float(np.float32(x))
    assert k["Adam/learning_rate"] == f32(1e-4) and k["Adam_1/learning_rate"] == f32(1e-3)
    assert k["Adam/beta1"] == f32(0.9) and k["Adam/beta2"] == f32(0.999)
    assert k["Adam/epsilon"] == f32(1e-8)
    assert k["Mul_2/y"] == f32(0.001) and k["Mul_3/y"] == f32(0.999)  # tau, 1 - tau
    assert k["Mul/y"] == 3.0  # InvertedPendulum action_scale
    assert k["gradients_1/MeanSquare/Square_grad/mul/x"] == 2.0
    assert k["FullyConnected_2/W/Initializer/random_uniform/max"] == f32(0.003)
    assert meta["op_histogram"]["ApplyAdam"] == 13
    assert all(d == "/job:ps/task:0" for d in meta["apply_adam_devices"].values())


def _ckpt_params(npz):
    z = np.load(npz)
    get = lambda names, keys: {k: z[n].astype(np.float64) for k, n in zip(keys, names)}
    return {"actor": get(O.CKPT_ACTOR, O.ACTOR_KEYS), "actor_t": get(O.CKPT_ACTOR_T, O.ACTOR_KEYS),
            "critic": get(O.CKPT_CRITIC, O.CRITIC_KEYS),
            "critic_t": get(O.CKPT_CRITIC_T, O.CRITIC_KEYS)}, z


def test_checkpoint_fixtures_decode():
    p, z = _ckpt_params(os.path.join(GOLD, "ip_model1410.npz"))
    assert p["actor"]["W1"].shape == (4, 128) and p["actor"]["W2"].shape == (128, 200)
    assert p["critic"]["Wh"].shape == (256, 200) and p["critic"]["Wo"].shape == (200, 1)
    # trained policy is bounded by action_scale = 3 and finite
    s = np.random.default_rng(0).standard_normal((32, 4))
    mu = O.actor_forward(p["actor"], s, 3.0)[3]
    assert np.all(np.abs(mu) <= 3.0) and np.all(np.isfinite(mu))
    q = O.critic_forward(p["critic"], s, mu)[3]
    assert np.all(np.isfinite(q))
    # MountainCar: 48/64 widths, Adam powers imply t ~ 45k steps
    pm, zm = _ckpt_params(os.path.join(GOLD, "mc_model120.npz"))
    assert pm["actor"]["W1"].shape == (2, 48) and pm["critic"]["Wh"].shape == (96, 128)
    b2p = float(zm["beta2_power_1"])
    t = np.log(b2p) / np.log(np.float32(0.999)) - 1
    assert 45000 < t < 46000
    # Adam second moments are non-negative; the m/v slots exist for every online var
    for n in O.CKPT_ACTOR + O.CKPT_CRITIC:
        assert (zm[n + "/Adam_1"] >= 0).all() and zm[n + "/Adam"].shape == zm[n].shape


def test_learner_step_fp32_tracks_fp64():
    """The fp32 restatement (TF's precision) stays within the parity
    tolerance of the fp64 restatement over several steps."""
    S, A, H1, H2, B = 4, 1, 32, 48, 64
    a, c = O.init_params(S, A, H1, H2, seed=5)
    at, ct = O.init_params(S, A, H1, H2, seed=6)
    params = {"actor": a, "actor_t": at, "critic": c, "critic_t": ct}
    L64 = O.Learner(S, A, H1, H2, 3.0, dtype=np.float64, params=params)
    L32 = O.Learner(S, A, H1, H2, 3.0, dtype=np.float32, params=params)
    rng = np.random.default_rng(0)
    for _ in range(5):
        s, s2 = rng.standard_normal((B, S)), rng.standard_normal((B, S))
        act = rng.uniform(-3, 3, (B, A))
        r, t = rng.standard_normal(B), rng.random(B) < 0.1
        o64 = L64.step(s, act, r, t, s2)
        o32 = L32.step(s, act, r, t, s2)
        np.testing.assert_allclose(o32["q"], o64["q"], rtol=1e-5, atol=1e-6)
    for net in ("actor", "critic", "actor_t", "critic_t"):
        for k, v in L64.state()[net].items():
            v32 = L32.state()[net][k]
            assert np.max(np.abs(v32 - v)) <= 1e-4 * max(np.max(np.abs(v)), 1e-3), (net, k)


def test_flops_formula():
    assert O.flops_per_step(64, 16, 1024, 1024, 4096, survey=True) == pytest.approx(142.46e9,
                                                                                     rel=1e-4)


def test_bench_flop_accounting_matches_oracle():
    """bench.py counts FLOP with distributed_ddpg_amd.flops; it must agree with
    the oracle's count."""
    from distributed_ddpg_amd.flops import flops_per_step as F
    for args in [(64, 16, 1024, 1024, 4096), (376, 17, 2048, 2048, 4096), (4, 1, 128, 200, 64)]:
        for kw in ({}, {"survey": True}, {"tf_recompute": True}):
            assert F(*args, **kw) == O.flops_per_step(*args, **kw)
