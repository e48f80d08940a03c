"""Pin the oracle to the reference's own TF graph.

tests/golden/graph_ip1410.npz holds a 3-step learner trajectory produced by
EXECUTING the reference's InvertedPendulum MetaGraphDef (model-1410.meta,
TF 1.3) from its own checkpoint (weights, targets, Adam slots, beta powers;
see make_graph_fixtures.py / tfgraph.py).  The oracle's restatement of
networks.py / ddpg.py:86-113, started from the same state and fed the same
batches, must reproduce every intermediate (target Q, TD target, pre-update Q,
loss, a_outs, dQ/da), every gradient an ApplyAdam consumed, and the final
weights / targets / Adam slots / beta powers.  Fixture arrays are stored as
float32, so the bar is a few float32 ulps (rel 1e-6); a wiring difference
(wrong operand, missing grad_ys sign, post- vs pre-update critic) is O(1).

The kernel FORMULAS (Elu, EluGrad, TanhGrad, ApplyAdam) are restated in both
the interpreter and the oracle; this pins the graph wiring, not TF's kernels.
"""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")
TOL = 1e-6


def rel(x, ref):
    x = np.asarray(x, np.float64)
    ref = np.asarray(ref, np.float64).reshape(x.shape)
    return float(np.max(np.abs(x - ref)) / max(np.max(np.abs(ref)), 1e-30))


def load_fixture_learner(O, dtype=np.float64):
    """Oracle Learner at the fixture's initial state (model-1410 + its Adam slots)."""
    z = np.load(os.path.join(GOLD, "graph_ip1410.npz"))
    w = np.load(os.path.join(GOLD, "ip_model1410.npz"))
    get = lambda names, keys: {k: w[n] for k, n in zip(keys, names)}
    p = {"actor": get(O.CKPT_ACTOR, O.ACTOR_KEYS), "actor_t": get(O.CKPT_ACTOR_T, O.ACTOR_KEYS),
         "critic": get(O.CKPT_CRITIC, O.CRITIC_KEYS),
         "critic_t": get(O.CKPT_CRITIC_T, O.CRITIC_KEYS)}
    L = O.Learner(4, 1, 128, 200, 3.0, dtype=dtype, params=p, init_blend=False)
    for opt, names, keys, sfx in ((L.actor_opt, O.CKPT_ACTOR, O.ACTOR_KEYS, ""),
                                  (L.critic_opt, O.CKPT_CRITIC, O.CRITIC_KEYS, "_1")):
        for k, n in zip(keys, names):
            opt.m[k] = z["init/%s/Adam" % n].astype(dtype)
            opt.v[k] = z["init/%s/Adam_1" % n].astype(dtype)
        opt.b1p = dtype(z["init/beta1_power" + sfx])
        opt.b2p = dtype(z["init/beta2_power" + sfx])
    return L, p, z


def test_oracle_reproduces_reference_graph_trajectory():
    from oracle import ddpg_oracle as O
    L, _, z = load_fixture_learner(O)
    for step in range(3):
        p = "step%d/" % step
        out = L.step(z[p + "s"], z[p + "a"], z[p + "r"], z[p + "t"], z[p + "s2"])
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
