"""GPU parity: the HIP path (through the C-ABI) vs the CPU oracle.

Tolerances (BASELINE.json north_star), measured as max|x - ref| / max|ref|
over each tensor:
  forward outputs                          1e-5
  gradients / parameters / Adam slots      1e-4 (fp32), after N steps
  soft update                              bit-exact (same fp32 ops as TF)
  replay indices / gathered rows           bit-exact
The oracle runs in float64 on the same fp32 inputs and weights.

Multi-step fused runs: Adam normalises every gradient element to ~lr, so
elements whose gradient is a near-cancelling fp32 sum carry fp32 rounding
straight into the parameter.  A TF-semantics fp32 restatement (the oracle in
float32, i.e. what the reference's TF 1.3 CPU path computes) drifts from fp64
by up to ~7e-5 on such tensors after 4 steps.  The multi-step bar is therefore
  max-rel  <= max(1e-4, 3 x the fp32 restatement's own max-rel drift), and
  norm-rel (||x - ref||_2 / ||ref||_2) <= 1e-5.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")

FWD_TOL = 1e-5
GRAD_TOL = 1e-4


def rel(x, ref):
    x = np.asarray(x, np.float64)
    ref = np.asarray(ref, np.float64)
    assert x.shape == ref.shape, (x.shape, ref.shape)
    den = max(np.max(np.abs(ref)), 1e-30)
    return float(np.max(np.abs(x - ref)) / den)


@pytest.fixture(scope="module")
def O():
    from oracle import ddpg_oracle
    return ddpg_oracle


@pytest.fixture(scope="module")
def dd():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    import distributed_ddpg_amd.networks as nets
    return nets


CONFIGS = {
    # name: S, A, H1, H2, scale, B, source  (critic widths in CRITIC_W when they differ)
    "ip": (4, 1, 128, 200, 3.0, 64, "ip_model1410"),
    # C2 at the reference's default batch (parameters.py:11)
    "ip256": (4, 1, 128, 200, 3.0, 256, "ip_model1410"),
    "mc": (2, 1, 48, 64, 1.0, 64, "mc_model120"),
    "odd": (5, 3, 40, 72, 2.0, 37, None),
    "wide": (64, 16, 1024, 1024, 1.0, 256, None),
    # S > 64: the first layers on the GEMMs, not thin_k
    "wides": (200, 16, 1024, 1024, 1.0, 256, None),
}
# the MountainCar checkpoint's critic is 48/128 while its actor is 48/64
CRITIC_W = {"mc": (48, 128)}


def cw(name):
    S, A, H1, H2 = CONFIGS[name][:4]
    return CRITIC_W.get(name, (H1, H2))


def _params(O, name):
    S, A, H1, H2, scale, B, src = CONFIGS[name]
    if src:
        z = np.load(os.path.join(GOLD, src + ".npz"))
        get = lambda names, keys: {k: z[n].astype(np.float32) for k, n in zip(keys, names)}
        p = {"actor": get(O.CKPT_ACTOR, O.ACTOR_KEYS), "actor_t": get(O.CKPT_ACTOR_T, O.ACTOR_KEYS),
             "critic": get(O.CKPT_CRITIC, O.CRITIC_KEYS),
             "critic_t": get(O.CKPT_CRITIC_T, O.CRITIC_KEYS)}
        return p, z
    a, c = O.init_params(S, A, H1, H2, seed=11)
    at, ct = O.init_params(S, A, H1, H2, seed=12)
    assert name not in CRITIC_W
    # larger-than-init weights so every branch (elu < 0, tanh saturation) is exercised
    rng = np.random.default_rng(3)
    for d in (a, c, at, ct):
        for k in d:
            d[k] = (d[k] + rng.standard_normal(d[k].shape).astype(np.float32) * 0.05).astype(
                np.float32)
    return {"actor": a, "actor_t": at, "critic": c, "critic_t": ct}, None


def _session(dd, O, name, p, batch_max=4096):
    S, A, H1, H2, scale, B, _ = CONFIGS[name]
    from distributed_ddpg_amd import _lib
    dd.reset_default_graph()
    actor = dd.ActorNetwork(S, A, scale, 1e-4, 1e-3, None, h1=H1, h2=H2)
    CH1, CH2 = cw(name)
    critic = dd.CriticNetwork(S, A, 1e-3, 1e-3, actor.get_num_trainable_vars(), None, h1=CH1,
                              h2=CH2)
    sess = dd.Session(batch_max=batch_max)
    actor.set_session(sess)
    critic.set_session(sess)
    sess.set_params(_lib.ACTOR, [p["actor"][k] for k in O.ACTOR_KEYS])
    sess.set_params(_lib.ACTOR_TARGET, [p["actor_t"][k] for k in O.ACTOR_KEYS])
    sess.set_params(_lib.CRITIC, [p["critic"][k] for k in O.CRITIC_KEYS])
    sess.set_params(_lib.CRITIC_TARGET, [p["critic_t"][k] for k in O.CRITIC_KEYS])
    return sess, actor, critic


def _batch(name, seed=0, B=None):
    S, A, H1, H2, scale, B0, _ = CONFIGS[name]
    B = B or B0
    rng = np.random.default_rng(seed)
    s = rng.standard_normal((B, S)).astype(np.float32)
    a = (rng.uniform(-1, 1, (B, A)) * scale).astype(np.float32)
    return s, a, rng


def normrel(x, ref):
    x = np.asarray(x, np.float64).ravel()
    ref = np.asarray(ref, np.float64).ravel()
    return float(np.linalg.norm(x - ref) / max(np.linalg.norm(ref), 1e-30))


def assert_steps_close(v, ref64, ref32, what):
    floor = rel(ref32.reshape(v.shape), ref64.reshape(v.shape))
    err = rel(v, ref64.reshape(v.shape))
    assert err <= max(GRAD_TOL, 3 * floor), (what, err, floor)
    assert normrel(v, ref64) <= 1e-5, (what, normrel(v, ref64))


def f64(d):
    return {k: v.astype(np.float64) for k, v in d.items()}


@pytest.mark.parametrize("name", list(CONFIGS))
def test_forward_parity(dd, O, name):
    S, A, H1, H2, scale, B, _ = CONFIGS[name]
    p, _ = _params(O, name)
    sess, actor, critic = _session(dd, O, name, p)
    s, a, _ = _batch(name)
    for Bq in (1, B):
        mu = actor.predict(s[:Bq])
        assert mu.dtype == np.float32 and mu.shape == (Bq, A)
        ref = O.actor_forward(f64(p["actor"]), s[:Bq].astype(np.float64), scale)[3]
        assert rel(mu, ref) < FWD_TOL
        mut = actor.predict_target(s[:Bq])
        assert rel(mut, O.actor_forward(f64(p["actor_t"]), s[:Bq].astype(np.float64), scale)[3]) < FWD_TOL
        q = critic.predict(s[:Bq], a[:Bq])
        assert q.shape == (Bq, 1)
        assert rel(q, O.critic_forward(f64(p["critic"]), s[:Bq].astype(np.float64),
                                       a[:Bq].astype(np.float64))[3]) < FWD_TOL
        qt = critic.predict_target(s[:Bq], a[:Bq])
        assert rel(qt, O.critic_forward(f64(p["critic_t"]), s[:Bq].astype(np.float64),
                                        a[:Bq].astype(np.float64))[3]) < FWD_TOL
    sess.close()


@pytest.mark.parametrize("name", ["ip", "wide"])
def test_forward_methods_any_batch(dd, O, name):
    """Forward-only methods take any batch, as a TF feed does: B = 0 returns
    empty [0, A] / [0, 1] arrays, and a batch past the session's batch_max
    runs in batch_max-row pieces -- within the forward bar of the oracle, and
    equal, row for row, to the same rows asked for in one call of their own
    size.  Training calls keep 1 <= B <= batch_max (their batch statistics
    cannot be split): B = 0 and B = batch_max + 1 raise ValueError."""
    S, A, H1, H2, scale, B, _ = CONFIGS[name]
    p, _ = _params(O, name)
    sess, actor, critic = _session(dd, O, name, p, batch_max=B)
    s, a, _ = _batch(name, seed=5, B=2 * B + 37)
    assert actor.predict(s[:0]).shape == (0, A)
    assert actor.predict_target(s[:0]).shape == (0, A)
    assert critic.predict(s[:0], a[:0]).shape == (0, 1)
    assert critic.action_gradients(s[:0], a[:0])[0].shape == (0, A)
    s64, a64 = s.astype(np.float64), a.astype(np.float64)
    mu = actor.predict(s)
    assert mu.shape == (2 * B + 37, A)
    assert rel(mu, O.actor_forward(f64(p["actor"]), s64, scale)[3]) < FWD_TOL
    mut = actor.predict_target(s)
    assert rel(mut, O.actor_forward(f64(p["actor_t"]), s64, scale)[3]) < FWD_TOL
    q = critic.predict(s, a)
    assert rel(q, O.critic_forward(f64(p["critic"]), s64, a64)[3]) < FWD_TOL
    qt = critic.predict_target(s, a)
    assert rel(qt, O.critic_forward(f64(p["critic_t"]), s64, a64)[3]) < FWD_TOL
    (da,) = critic.action_gradients(s, a)
    assert rel(da, O.critic_action_grads(f64(p["critic"]), s64, a64)) < GRAD_TOL
    # the last piece (37 rows) equals the same rows in a call of their own
    assert np.array_equal(mu[2 * B:], actor.predict(s[2 * B:]))
    assert np.array_equal(q[2 * B:], critic.predict(s[2 * B:], a[2 * B:]))
    y = np.zeros((B + 1, 1), np.float32)
    for n in (0, B + 1):
        with pytest.raises(ValueError, match="outside"):
            critic.train(s[:n], a[:n], y[:n])
        with pytest.raises(ValueError, match="outside"):
            actor.train(s[:n], a[:n])
    sess.close()


@pytest.mark.parametrize("name", list(CONFIGS))
def test_train_methods_parity(dd, O, name):
    """critic.train -> action_gradients -> actor.train, 3 rounds, vs oracle."""
    from distributed_ddpg_amd import _lib
    S, A, H1, H2, scale, B, _ = CONFIGS[name]
    p, _ = _params(O, name)
    sess, actor, critic = _session(dd, O, name, p)
    L = O.Learner(S, A, H1, H2, scale, actor_lr=1e-4, critic_lr=1e-3, tau=1e-3,
                  dtype=np.float64, params=p, init_blend=False, CH1=cw(name)[0], CH2=cw(name)[1])
    for it in range(3):
        s, a, rng = _batch(name, seed=10 + it)
        y = rng.standard_normal((B, 1)).astype(np.float32)
        q, none, loss = critic.train(s, a, y)
        assert none is None and q.shape == (B, 1) and q.dtype == np.float32
        q_ref, loss_ref, _ = L.critic_train(s.astype(np.float64), a.astype(np.float64),
                                            y.astype(np.float64))
        assert rel(q, q_ref) < FWD_TOL
        assert abs(float(loss) - loss_ref) <= GRAD_TOL * abs(loss_ref)
        a_out = actor.predict(s)
        a_ref = L.actor_predict(s.astype(np.float64))
        assert rel(a_out, a_ref) < FWD_TOL
        (da,) = critic.action_gradients(s, a_out)
        da_ref = L.action_gradients(s.astype(np.float64), a_out.astype(np.float64))
        assert rel(da, da_ref) < GRAD_TOL
        actor.train(s, da)
        L.actor_train(s.astype(np.float64), da.astype(np.float64))
    got_c = sess.get_params(_lib.CRITIC)
    got_a = sess.get_params(_lib.ACTOR)
    for k, v in zip(O.CRITIC_KEYS, got_c):
        assert rel(v, L.critic[k].reshape(v.shape)) < GRAD_TOL, ("critic", k)
    for k, v in zip(O.ACTOR_KEYS, got_a):
        assert rel(v, L.actor[k].reshape(v.shape)) < GRAD_TOL, ("actor", k)
    for which, opt, keys in ((_lib.CRITIC_ADAM_M, L.critic_opt.m, O.CRITIC_KEYS),
                             (_lib.CRITIC_ADAM_V, L.critic_opt.v, O.CRITIC_KEYS),
                             (_lib.ACTOR_ADAM_M, L.actor_opt.m, O.ACTOR_KEYS),
                             (_lib.ACTOR_ADAM_V, L.actor_opt.v, O.ACTOR_KEYS)):
        for k, v in zip(keys, sess.get_params(which)):
            assert rel(v, opt[k].reshape(v.shape)) < GRAD_TOL, (which, k)
    b1p, b2p = sess.get_adam_powers(1)
    assert b1p == np.float32(0.9) ** 4 or abs(b1p - 0.9 ** 4) < 1e-7
    assert abs(b2p - 0.999 ** 4) < 1e-6
    sess.close()


def test_soft_update_bitexact(dd, O):
    from distributed_ddpg_amd import _lib
    p, _ = _params(O, "odd")
    sess, actor, critic = _session(dd, O, "odd", p)
    for _ in range(2):
        actor.update_target_network()
    critic.update_target_network()
    tau, omt = np.float32(0.001), np.float32(0.999)
    exp_a = {k: p["actor_t"][k].copy() for k in O.ACTOR_KEYS}
    for _ in range(2):
        exp_a = {k: (p["actor"][k] * tau + exp_a[k] * omt).astype(np.float32) for k in exp_a}
    exp_c = {k: (p["critic"][k] * tau + p["critic_t"][k] * omt).astype(np.float32)
             for k in O.CRITIC_KEYS}
    for k, v in zip(O.ACTOR_KEYS, sess.get_params(_lib.ACTOR_TARGET)):
        assert np.array_equal(v, exp_a[k].reshape(v.shape)), k
    for k, v in zip(O.CRITIC_KEYS, sess.get_params(_lib.CRITIC_TARGET)):
        assert np.array_equal(v, exp_c[k].reshape(v.shape)), k
    sess.close()


def test_mc_checkpoint_adam_resume(dd, O):
    """Resume from the reference's MountainCar checkpoint mid-run (t ~ 45k
    Adam steps, non-trivial bias correction): restore weights, Adam slots and
    beta powers, do one critic/actor update, compare with the oracle."""
    from distributed_ddpg_amd import _lib
    p, z = _params(O, "mc")
    S, A, H1, H2, scale, B, _ = CONFIGS["mc"]
    sess, actor, critic = _session(dd, O, "mc", p)
    slots = lambda names, suf: [z[n + suf] for n in names]
    sess.set_params(_lib.ACTOR_ADAM_M, slots(O.CKPT_ACTOR, "/Adam"))
    sess.set_params(_lib.ACTOR_ADAM_V, slots(O.CKPT_ACTOR, "/Adam_1"))
    sess.set_params(_lib.CRITIC_ADAM_M, slots(O.CKPT_CRITIC, "/Adam"))
    sess.set_params(_lib.CRITIC_ADAM_V, slots(O.CKPT_CRITIC, "/Adam_1"))
    sess.set_adam_powers(0, float(z["beta1_power"]), float(z["beta2_power"]))
    sess.set_adam_powers(1, float(z["beta1_power_1"]), float(z["beta2_power_1"]))
    L = O.Learner(S, A, H1, H2, scale, dtype=np.float64, params=p, init_blend=False,
                  CH1=cw("mc")[0], CH2=cw("mc")[1])
    for net, names in ((L.actor_opt, O.CKPT_ACTOR), (L.critic_opt, O.CKPT_CRITIC)):
        keys = O.ACTOR_KEYS if names is O.CKPT_ACTOR else O.CRITIC_KEYS
        for k, n in zip(keys, names):
            net.m[k] = z[n + "/Adam"].astype(np.float64)
            net.v[k] = z[n + "/Adam_1"].astype(np.float64)
    L.actor_opt.b1p, L.actor_opt.b2p = np.float64(z["beta1_power"]), np.float64(z["beta2_power"])
    L.critic_opt.b1p, L.critic_opt.b2p = (np.float64(z["beta1_power_1"]),
                                          np.float64(z["beta2_power_1"]))
    s, a, rng = _batch("mc", seed=5)
    y = rng.standard_normal((B, 1)).astype(np.float32)
    critic.train(s, a, y)
    L.critic_train(s.astype(np.float64), a.astype(np.float64), y.astype(np.float64))
    da = rng.standard_normal((B, A)).astype(np.float32)
    actor.train(s, da)
    L.actor_train(s.astype(np.float64), da.astype(np.float64))
    for k, v in zip(O.CRITIC_KEYS, sess.get_params(_lib.CRITIC)):
        assert rel(v, L.critic[k].reshape(v.shape)) < GRAD_TOL, k
    for k, v in zip(O.ACTOR_KEYS, sess.get_params(_lib.ACTOR)):
        assert rel(v, L.actor[k].reshape(v.shape)) < GRAD_TOL, k
    sess.close()


def _fill(rb, S, A, n, scale, seed):
    rng = np.random.default_rng(seed)
    s = rng.standard_normal((n, S)).astype(np.float32)
    s2 = rng.standard_normal((n, S)).astype(np.float32)
    a = (rng.uniform(-1, 1, (n, A)) * scale).astype(np.float32)
    r = rng.standard_normal(n).astype(np.float32)
    t = rng.random(n) < 0.05
    rb.add_batch(s, a, r, t, s2)
    return s, a, r, t, s2


def test_replay_device_sample_bitexact(dd):
    """Device ring + host sampler reproduce the reference's index streams
    (golden fixture cases) and return exactly the inserted rows."""
    import json
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    z = np.load(os.path.join(GOLD, "replay_indices.npz"))
    cases = {c["name"]: c for c in json.loads(bytes(z["__cases__"]).decode())}
    for name in ("survey_prewrap", "survey_postwrap", "interleaved_wrap", "count_lt_batch",
                 "pool_branch_b256", "full_1e6_b4096"):
        c = cases[name]
        rb = ReplayBuffer(c["capacity"], c["seed"])
        total, j = 0, 0
        for op, n in c["ops"]:
            if op == "add":
                ids = np.arange(total, total + n)
                rb.add_batch(ids[:, None].astype(np.float32) % 1e7, np.zeros((n, 1), np.float32),
                             (ids * 0.5).astype(np.float32), ids % 7 == 0,
                             (ids[:, None] % 1e7).astype(np.float32))
                total += n
            else:
                s, a, r, t, s2, idx = rb.sample_batch(n, return_indices=True)
                exp = z["%s__%d" % (name, j)]
                ins = (total - rb.size()) + idx
                assert np.array_equal(ins, exp), name
                assert np.array_equal(s[:, 0], (exp % 10_000_000).astype(np.float64)), name
                assert np.array_equal(r, (exp * 0.5).astype(np.float32).astype(np.float64))
                assert np.array_equal(t, exp % 7 == 0)
                assert s.dtype == np.float64 and a.dtype == np.float32 and t.dtype == bool
                j += 1


@pytest.mark.parametrize("name", ["ip", "ip256", "odd", "wide"])
def test_fused_learner_step_parity(dd, O, name):
    """ddpg_learner_step (sample -> gather -> whole update on device) vs the
    oracle's ddpg.py:86-113 sequence on the same sampled rows, 4 steps."""
    import random
    from distributed_ddpg_amd import _lib
    from distributed_ddpg_amd.learner import FusedLearner
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    S, A, H1, H2, scale, B, _ = CONFIGS[name]
    p, _ = _params(O, name)
    sess, actor, critic = _session(dd, O, name, p)
    rb = ReplayBuffer(5000, 1234)
    rows = _fill(rb, S, A, 3000, scale, seed=2)
    fl = FusedLearner(sess, rb, B)
    L = O.Learner(S, A, H1, H2, scale, dtype=np.float64, params=p, init_blend=False)
    L32 = O.Learner(S, A, H1, H2, scale, dtype=np.float32, params=p, init_blend=False)
    ref_rng = random.Random(1234)  # the reference's global RNG after random.seed(1234)
    for it in range(4):
        idx = np.array(ref_rng.sample(range(3000), B))
        qmax, loss = fl.step(stats=True)
        s, a, r, t, s2 = (x[idx] for x in rows)
        out = L.step(s, a, r, t, s2)
        L32.step(s, a, r, t, s2)
        assert abs(qmax - float(np.max(out["q"]))) <= FWD_TOL * max(1.0, abs(np.max(out["q"]))) * 10
        assert abs(loss - float(out["loss"])) <= GRAD_TOL * abs(float(out["loss"]))
    for which, net, keys in ((_lib.ACTOR, "actor", O.ACTOR_KEYS),
                             (_lib.CRITIC, "critic", O.CRITIC_KEYS),
                             (_lib.ACTOR_TARGET, "actor_t", O.ACTOR_KEYS),
                             (_lib.CRITIC_TARGET, "critic_t", O.CRITIC_KEYS)):
        for k, v in zip(keys, sess.get_params(which)):
            assert_steps_close(v, L.state()[net][k], L32.state()[net][k], (net, k))
    q_sum, l_sum, n = fl.read_stats()
    assert n == 4
    sess.close()


def _fused_state(sess):
    from distributed_ddpg_amd import _lib
    return [sess.get_params(w) for w in (_lib.ACTOR, _lib.CRITIC, _lib.ACTOR_TARGET,
                                         _lib.CRITIC_TARGET, _lib.ACTOR_ADAM_M,
                                         _lib.ACTOR_ADAM_V, _lib.CRITIC_ADAM_M,
                                         _lib.CRITIC_ADAM_V)]


@pytest.mark.parametrize("name", ["ip", "wide"])
def test_rejected_calls_leave_state_unchanged(dd, O, name):
    """Error behaviour of the fused step (the reference's feed would raise TF's
    InvalidArgumentError): a batch past batch_max, a replay of other dims, a
    replay holding fewer rows than the batch, a parameter upload of the wrong
    size and a wrong parameter-set id each raise DDPGError, and none of them
    moves anything -- the replay's sampler, the parameters, the Adam state:
    the session's next two steps equal, bit for bit, those of a session that
    never saw the rejected calls (small path "ip", GEMM path "wide")."""
    from distributed_ddpg_amd import _lib
    from distributed_ddpg_amd.learner import FusedLearner
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    S, A, H1, H2, scale, B, _ = CONFIGS[name]
    p, _ = _params(O, name)
    runs = []
    for bad in (False, True):
        sess, actor, critic = _session(dd, O, name, p, batch_max=B)
        rb = ReplayBuffer(5000, 1234)
        _fill(rb, S, A, 3000, scale, seed=2)
        if bad:
            with pytest.raises(_lib.DDPGError, match="batch"):
                FusedLearner(sess, rb, B + 1).step()
            other = ReplayBuffer(500, 99)
            _fill(other, S + 1, A, 400, scale, seed=3)
            with pytest.raises(_lib.DDPGError, match="replay dims"):
                FusedLearner(sess, other, B).step()
            few = ReplayBuffer(500, 7)
            _fill(few, S, A, B - 1, scale, seed=4)
            with pytest.raises(_lib.DDPGError, match="rows < batch"):
                FusedLearner(sess, few, B).step()
            w = sess.get_params(_lib.ACTOR)
            with pytest.raises(_lib.DDPGError):
                sess.set_params(_lib.ACTOR, w[:-1])
            with pytest.raises(_lib.DDPGError):
                sess.set_params(99, w)
        fl = FusedLearner(sess, rb, B)
        st = [fl.step(stats=True) for _ in range(2)]
        runs.append((st, _fused_state(sess), fl.read_stats()))
        sess.close()
    (st0, s0, a0), (st1, s1, a1) = runs
    assert st0 == st1 and a0 == a1
    for x, y in zip(s0, s1):
        for u, v in zip(x, y):
            assert np.array_equal(u, v)


def test_batch_4096_wide_step_properties(dd, O):
    """Full C3 shape (S=64, A=16, 1024/1024, B=4096): one fused step equals
    the oracle step on the same rows (fp64 oracle at full size)."""
    import random
    from distributed_ddpg_amd import _lib
    from distributed_ddpg_amd.learner import FusedLearner
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    S, A, H1, H2, scale = 64, 16, 1024, 1024, 1.0
    B = 4096
    p, _ = _params(O, "wide")
    sess, actor, critic = _session(dd, O, "wide", p, batch_max=B)
    rb = ReplayBuffer(20000, 77)
    rows = _fill(rb, S, A, 20000, scale, seed=9)
    fl = FusedLearner(sess, rb, B)
    idx = np.array(random.Random(77).sample(range(20000), B))
    fl.step()
    L = O.Learner(S, A, H1, H2, scale, dtype=np.float64, params=p, init_blend=False)
    L.step(*(x[idx] for x in rows))
    for which, ref, keys in ((_lib.ACTOR, L.actor, O.ACTOR_KEYS),
                             (_lib.CRITIC, L.critic, O.CRITIC_KEYS)):
        for k, v in zip(keys, sess.get_params(which)):
            assert rel(v, ref[k].reshape(v.shape)) < GRAD_TOL, (which, k)
    sess.close()


@pytest.mark.parametrize("name", ["ip", "wide"])
def test_graph_replay_matches_eager(dd, O, monkeypatch, name):
    """The hipGraph-replayed fused step is bit-identical to eager launches
    (all kernels are deterministic: no atomics in any reduction).  Variants:
    the default issue policy (small path: every step eager; large path: graph
    replay), DDPG_GRAPH_AUTO=1 (graph replay when the previous step has
    finished, eager launches when it is still running: steps without stats
    are not synchronised, so this run mixes both), graph replay only
    (DDPG_GRAPH_AUTO=0) and eager only (DDPG_GRAPH=0)."""
    from distributed_ddpg_amd import _lib
    from distributed_ddpg_amd.learner import FusedLearner
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    S, A, H1, H2, scale, B, _ = CONFIGS[name]
    p, _ = _params(O, name)
    out = []
    for graph, auto in (("1", "2"), ("1", "1"), ("1", "0"), ("0", "1")):
        monkeypatch.setenv("DDPG_GRAPH", graph)
        monkeypatch.setenv("DDPG_GRAPH_AUTO", auto)
        sess, actor, critic = _session(dd, O, name, p)
        rb = ReplayBuffer(2000, 99)
        _fill(rb, S, A, 1500, scale, seed=4)
        fl = FusedLearner(sess, rb, B)
        stats = [fl.step(stats=(i % 3 == 0)) for i in range(7)]
        out.append((stats, [sess.get_params(w) for w in (_lib.ACTOR, _lib.CRITIC,
                                                         _lib.ACTOR_TARGET, _lib.CRITIC_TARGET)],
                    sess.get_adam_powers(0), sess.get_adam_powers(1)))
        sess.close()
    s0, p0, a0, c0 = out[-1]
    for s1, p1, a1, c1 in out[:-1]:
        assert s1 == s0 and a1 == a0 and c1 == c0
        for x, y in zip(p1, p0):
            for u, v in zip(x, y):
                assert np.array_equal(u, v)


# ---------------------------------------------------------------------- bf16
# bf16 GEMM operands (v_mfma_f32_32x32x16_bf16), fp32 accumulation, fp32
# master weights / Adam / epilogues.  Stated bf16 tolerances (vs the fp64
# oracle, max-rel per tensor): forward outputs 2e-2; dQ/da 5e-2; parameters
# after 3 fused steps 2e-2 (Adam moves every weight by ~lr per step, so the
# parameter error stays a fraction of lr even with bf16 gradients).
BF16_FWD_TOL, BF16_DA_TOL, BF16_PARAM_TOL = 2e-2, 5e-2, 2e-2


def _session_dtype(dd, O, name, p, dtype, batch_max=4096):
    S, A, H1, H2, scale, B, _ = CONFIGS[name]
    from distributed_ddpg_amd import _lib
    dd.reset_default_graph()
    actor = dd.ActorNetwork(S, A, scale, 1e-4, 1e-3, None, h1=H1, h2=H2)
    critic = dd.CriticNetwork(S, A, 1e-3, 1e-3, 10, None, h1=H1, h2=H2)
    sess = dd.Session(batch_max=batch_max, dtype=dtype)
    actor.set_session(sess)
    critic.set_session(sess)
    sess.set_params(_lib.ACTOR, [p["actor"][k] for k in O.ACTOR_KEYS])
    sess.set_params(_lib.ACTOR_TARGET, [p["actor_t"][k] for k in O.ACTOR_KEYS])
    sess.set_params(_lib.CRITIC, [p["critic"][k] for k in O.CRITIC_KEYS])
    sess.set_params(_lib.CRITIC_TARGET, [p["critic_t"][k] for k in O.CRITIC_KEYS])
    return sess, actor, critic


def test_bf16_parity_and_kernel_use(dd, O):
    import random
    from distributed_ddpg_amd import _lib
    from distributed_ddpg_amd.learner import FusedLearner, Profile
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    S, A, H1, H2, scale, B, _ = CONFIGS["wide"]
    p, _ = _params(O, "wide")
    sess, actor, critic = _session_dtype(dd, O, "wide", p, "bf16")
    s, a, _ = _batch("wide", seed=21)
    mu = actor.predict(s)
    assert rel(mu, O.actor_forward(f64(p["actor"]), s.astype(np.float64), scale)[3]) < BF16_FWD_TOL
    q = critic.predict(s, a)
    assert rel(q, O.critic_forward(f64(p["critic"]), s.astype(np.float64),
                                   a.astype(np.float64))[3]) < BF16_FWD_TOL
    (da,) = critic.action_gradients(s, mu)
    assert rel(da, O.critic_action_grads(f64(p["critic"]), s.astype(np.float64),
                                         mu.astype(np.float64))) < BF16_DA_TOL
    rb = ReplayBuffer(5000, 1234)
    rows = _fill(rb, S, A, 3000, scale, seed=2)
    fl = FusedLearner(sess, rb, B)
    prof = Profile(sess)
    prof.enable(True)
    L = O.Learner(S, A, H1, H2, scale, dtype=np.float64, params=p, init_blend=False)
    ref_rng = random.Random(1234)
    for it in range(3):
        idx = np.array(ref_rng.sample(range(3000), B))
        fl.step()
        L.step(*(x[idx] for x in rows))
    keys = prof.read()
    prof.enable(False)
    assert any((k.startswith("gemm_s3_kernel") and "NP=1" in k) or
               (k.startswith("gemm_h") and "NP=1" in k) for k in keys), sorted(keys)
    for which, net, names in ((_lib.ACTOR, "actor", O.ACTOR_KEYS),
                              (_lib.CRITIC, "critic", O.CRITIC_KEYS)):
        for k, v in zip(names, sess.get_params(which)):
            assert rel(v, L.state()[net][k].reshape(v.shape)) < BF16_PARAM_TOL, (net, k)
    sess.close()


@pytest.mark.parametrize("name", ["ip", "odd"])
def test_small_batch_path_matches_large_path(dd, O, monkeypatch, name):
    """The fused small-batch path (small_batch.h, 4 launches) and the
    large-batch GEMM path (DDPG_SMALL=0) agree after 4 steps (different
    summation order only), and both track the oracle."""
    from distributed_ddpg_amd import _lib
    from distributed_ddpg_amd.learner import FusedLearner, Profile
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    import random
    S, A, H1, H2, scale, B, _ = CONFIGS[name]
    p, _ = _params(O, name)
    # the oracle on the same rows (the replay's sampler = random.Random(5))
    L = O.Learner(S, A, H1, H2, scale, dtype=np.float64, params=p, init_blend=False)
    L32 = O.Learner(S, A, H1, H2, scale, dtype=np.float32, params=p, init_blend=False)
    ref_rng = random.Random(5)
    res = {}
    for small in ("1", "0"):
        monkeypatch.setenv("DDPG_SMALL", small)
        sess, actor, critic = _session(dd, O, name, p)
        rb = ReplayBuffer(4000, 5)
        rows = _fill(rb, S, A, 3000, scale, seed=8)
        if small == "1":
            for _ in range(4):
                idx = np.array(ref_rng.sample(range(3000), B))
                L.step(*(x[idx] for x in rows))
                L32.step(*(x[idx] for x in rows))
        fl = FusedLearner(sess, rb, B)
        prof = Profile(sess)
        prof.enable(True)
        st = [fl.step(stats=True) for _ in range(4)]
        keys = prof.read()
        prof.enable(False)
        assert any(k.startswith("sb_phase") for k in keys) == (small == "1"), sorted(keys)
        res[small] = (st, [sess.get_params(w) for w in (_lib.ACTOR, _lib.CRITIC,
                                                       _lib.ACTOR_TARGET, _lib.CRITIC_TARGET)],
                      sess.get_adam_powers(0), sess.get_adam_powers(1))
        sess.close()
    (s1, p1, a1, c1), (s0, p0, a0, c0) = res["1"], res["0"]
    assert a1 == a0 and c1 == c0
    for (q1, l1), (q0, l0) in zip(s1, s0):
        assert abs(q1 - q0) <= 1e-5 * max(1.0, abs(q0))
        assert abs(l1 - l0) <= 1e-4 * abs(l0)
    for x, y in zip(p1, p0):
        for u, v in zip(x, y):
            assert rel(u, v) < GRAD_TOL
    # and each path against the oracle
    nets = (("actor", O.ACTOR_KEYS), ("critic", O.CRITIC_KEYS), ("actor_t", O.ACTOR_KEYS),
            ("critic_t", O.CRITIC_KEYS))
    for params in (p1, p0):
        for (net, keys), vals in zip(nets, params):
            for k, v in zip(keys, vals):
                assert_steps_close(v, L.state()[net][k], L32.state()[net][k], (net, k))


@pytest.mark.parametrize("name", ["ip", "odd"])
def test_action_selection_single_launch(dd, O, name):
    """actor.predict at B = 1 (ddpg.py:68-70, the action-selection forward,
    SURVEY.md §8(f)1) is one sb_actor_predict launch (states in the kernel
    arguments, result written to pinned host memory) and matches the oracle;
    so is a small batch."""
    from distributed_ddpg_amd.learner import Profile
    S, A, H1, H2, scale, B, _ = CONFIGS[name]
    p, _ = _params(O, name)
    sess, actor, critic = _session(dd, O, name, p)
    s, _, _ = _batch(name)
    prof = Profile(sess)
    prof.enable(True)
    for lo, hi in ((0, 1), (1, 2), (5, 6), (0, 9)):
        for target, net in ((False, "actor"), (True, "actor_t")):
            mu = actor.predict_target(s[lo:hi]) if target else actor.predict(s[lo:hi])
            assert mu.dtype == np.float32 and mu.shape == (hi - lo, A)
            ref = O.actor_forward(f64(p[net]), s[lo:hi].astype(np.float64), scale)[3]
            assert rel(mu, ref) < FWD_TOL, (lo, hi, net)
    keys = prof.read()
    prof.enable(False)
    assert any(k.startswith("sb_actor_predict") for k in keys), sorted(keys)
    assert not any(k.startswith("gemm") for k in keys), sorted(keys)
    sess.close()


def test_saver_restores_reference_checkpoint_and_resumes(dd, O, tmp_path):
    """tf.train.Saver work-alike on a live session: restore
    the reference's MountainCar model-120 (ddpg.py:213-222), check every
    tensor and both beta-power pairs on the device, continue training one
    fused step from it (non-trivial Adam bias correction, t ~ 45k), and
    check that saving the untouched restored state reproduces TF's bytes."""
    from distributed_ddpg_amd import _lib, checkpoint as C
    from distributed_ddpg_amd.learner import FusedLearner
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    ref = os.path.join(GOLD, "ckpt", "model-120")
    p, _ = _params(O, "mc")
    sess, actor, critic = _session(dd, O, "mc", p)
    saver = C.Saver()
    t = saver.restore(sess, ref)
    for which, names in ((_lib.ACTOR, C.ACTOR), (_lib.CRITIC, C.CRITIC),
                         (_lib.ACTOR_TARGET, C.ACTOR_TARGET), (_lib.CRITIC_TARGET, C.CRITIC_TARGET),
                         (_lib.ACTOR_ADAM_V, [n + "/Adam_1" for n in C.ACTOR]),
                         (_lib.CRITIC_ADAM_M, [n + "/Adam" for n in C.CRITIC])):
        for n, v in zip(names, sess.get_params(which)):
            np.testing.assert_array_equal(v, t[n].reshape(v.shape))
    assert sess.get_adam_powers(1) == (float(t["beta1_power_1"]), float(t["beta2_power_1"]))
    out = saver.save(sess, str(tmp_path / "model"), global_step=120,
                     summary_values=[float(t[v]) for v in C.SUMMARY_VARS])
    for ext in (".index", ".data-00000-of-00001"):
        assert open(out + ext, "rb").read() == open(ref + ext, "rb").read(), ext
    # resume: one fused learner step from the restored state vs the oracle
    import random
    rb = ReplayBuffer(2000, 1234)
    rows = _fill(rb, 2, 1, 1000, 1.0, seed=4)
    L = O.Learner(2, 1, 48, 64, 1.0, dtype=np.float64, init_blend=False, CH1=48, CH2=128,
                  params={"actor": dict(zip(O.ACTOR_KEYS, [t[n] for n in C.ACTOR])),
                          "actor_t": dict(zip(O.ACTOR_KEYS, [t[n] for n in C.ACTOR_TARGET])),
                          "critic": dict(zip(O.CRITIC_KEYS, [t[n] for n in C.CRITIC])),
                          "critic_t": dict(zip(O.CRITIC_KEYS, [t[n] for n in C.CRITIC_TARGET]))})
    for opt, keys, names, sfx in ((L.actor_opt, O.ACTOR_KEYS, C.ACTOR, ""),
                                  (L.critic_opt, O.CRITIC_KEYS, C.CRITIC, "_1")):
        for k, n in zip(keys, names):
            opt.m[k] = t[n + "/Adam"].astype(np.float64)
            opt.v[k] = t[n + "/Adam_1"].astype(np.float64)
        opt.b1p = np.float64(t["beta1_power" + sfx])
        opt.b2p = np.float64(t["beta2_power" + sfx])
    idx = np.array(random.Random(1234).sample(range(1000), 64))
    FusedLearner(sess, rb, 64).step()
    L.step(*(x[idx] for x in rows))
    for which, net, names in ((_lib.ACTOR, "actor", O.ACTOR_KEYS),
                              (_lib.CRITIC, "critic", O.CRITIC_KEYS)):
        for k, v in zip(names, sess.get_params(which)):
            assert rel(v, L.state()[net][k].reshape(v.shape)) < GRAD_TOL, (net, k)
    sess.close()


def test_worker_driver_summaries_and_checkpoints(tmp_path):
    """The ddpg.py-compatible worker (episode loop on the fused path) writes
    the chief's TensorBoard scalars every episode (ddpg.py:118-125) and a
    checkpoint every valid_freq episodes (ddpg.py:262-264); continue_training
    restores the latest one (ddpg.py:213-222) and resumes its global_step."""
    from distributed_ddpg_amd import checkpoint as C, ddpg, summary as Sm
    from distributed_ddpg_amd.parameters import Parameters
    opt = Parameters()
    opt.batch_size, opt.rm_size, opt.valid_freq = 64, 20000, 2
    opt.summary_dir, opt.save_dir = str(tmp_path / "tboard"), str(tmp_path / "model")
    ddpg.run_worker(opt, 0, "synthetic", 3, 0)
    ev = [f for f in os.listdir(opt.summary_dir) if f.startswith("events.out.tfevents.")]
    assert len(ev) == 1
    sc = Sm.read_scalars(os.path.join(opt.summary_dir, ev[0]))
    assert [s for s, _ in sc["Reward"]] == [0, 1, 2]
    assert all(v >= 1.0 for _, v in sc["Reward"]) and len(sc["Value_Loss"]) == 3
    latest = C.latest_checkpoint(opt.save_dir)
    assert latest.endswith("model-1")
    t = C.read_bundle(latest)
    assert float(t["global_step"]) == 1.0 and len(t) == 62
    opt.continue_training = True
    opt.summary_dir = str(tmp_path / "tboard2")
    ddpg.run_worker(opt, 0, "synthetic", 1, 0)
    ev2 = os.listdir(opt.summary_dir)[0]
    assert [s for s, _ in Sm.read_scalars(os.path.join(opt.summary_dir, ev2))["Reward"]] == [1]
