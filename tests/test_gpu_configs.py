"""GPU parity at every BASELINE.json configuration, through the C-ABI.

  C1  MountainCar (S=2, A=1, scale 1) with the StandardScaler input path
      (ddpg.py:184-189, networks.py:65-69,164-168), B=64, at the code's 128/200
      and BASELINE's 400/300 widths; float64 replay rows.
  C2  InvertedPendulum at the reference default batch 256 (parameters.py:11)
      -- covered by CONFIGS["ip256"] in test_gpu_parity.py.
  C3  B=4096, 1024/1024: the gradient buffer and the Adam m / v slots after
      one fused step (m = 0.1 g, v = 0.001 g^2 on the first step).
  C4  data parallel: two world=2 contexts (ranks 0 and 1, no communicator) on
      one GPU run the product's slice of the global draw; their gradients and
      loss shares sum to the world=1 global-batch ones.
  C5  S=376, A=17, 2048/2048, B=4096, bf16 operands (stated bf16 bars).

Bars (max|x-ref|/max|ref| per tensor unless stated; oracle in float64 on the
fp32 values the device sees):
  forward 1e-5; gradients / parameters / Adam slots 1e-4 (fp32);
  bf16: forward 2e-2, dQ/da 5e-2, gradients norm-rel 3e-2, weight matrices (>= 64x64)
  2e-2 after one step and every parameter within 2 lr of the oracle.
"""
import os
import random

import numpy as np
import pytest

from test_gpu_parity import FWD_TOL, GRAD_TOL, f64, rel, normrel

pytestmark = pytest.mark.gpu


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


def _noisy_params(O, S, A, H1, H2, seed, amp=0.05):
    a, c = O.init_params(S, A, H1, H2, seed=seed)
    at, ct = O.init_params(S, A, H1, H2, seed=seed + 1)
    rng = np.random.default_rng(seed + 2)
    for d in (a, c, at, ct):
        for k in d:
            d[k] = (d[k] + rng.standard_normal(d[k].shape) * amp).astype(np.float32)
    return {"actor": a, "actor_t": at, "critic": c, "critic_t": ct}


def _open(dd, O, S, A, H1, H2, scale, p, batch_max, scaler=None, dtype="fp32", rank=0, world=1,
          critic_lr=1e-3):
    from distributed_ddpg_amd import _lib
    dd.reset_default_graph()
    actor = dd.ActorNetwork(S, A, scale, 1e-4, 1e-3, scaler, h1=H1, h2=H2)
    critic = dd.CriticNetwork(S, A, critic_lr, 1e-3, actor.get_num_trainable_vars(), scaler,
                              h1=H1, h2=H2)
    sess = dd.Session(batch_max=batch_max, dtype=dtype, rank=rank, world=world)
    actor.set_session(sess)
    critic.set_session(sess)
    sess.set_params(_lib.ACTOR, [p["actor"][k] for k in O.ACTOR_KEYS])
    sess.set_params(_lib.ACTOR_TARGET, [p["actor_t"][k] for k in O.ACTOR_KEYS])
    sess.set_params(_lib.CRITIC, [p["critic"][k] for k in O.CRITIC_KEYS])
    sess.set_params(_lib.CRITIC_TARGET, [p["critic_t"][k] for k in O.CRITIC_KEYS])
    return sess, actor, critic


def _rows(rng, n, S, A, scale, dtype=np.float32, lo=None, hi=None):
    if lo is None:
        s = rng.standard_normal((n, S))
        s2 = rng.standard_normal((n, S))
    else:
        s = rng.uniform(lo, hi, (n, S))
        s2 = rng.uniform(lo, hi, (n, S))
    a = (rng.uniform(-1, 1, (n, A)) * scale).astype(np.float32)
    r = rng.standard_normal(n)
    t = rng.random(n) < 0.05
    return s.astype(dtype), a, r.astype(dtype), t, s2.astype(dtype)


# ---------------------------------------------------------------- C1
MC_LOW, MC_HIGH = np.array([-1.2, -0.07]), np.array([0.6, 0.07])  # MountainCarContinuous obs box


@pytest.mark.parametrize("widths", [(128, 200), (400, 300)])
def test_mountaincar_scaler_parity(dd, O, widths):
    """The scaler is applied exactly once, in float64, on every path: the 1:1
    methods (host preprocess_input, as the reference) and the fused step
    (device gather from a float64 ring).  Created FusedLearner first: that is
    when the device scaler is uploaded."""
    from sklearn.preprocessing import StandardScaler
    from distributed_ddpg_amd import _lib
    from distributed_ddpg_amd.learner import FusedLearner
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    S, A, scale, B = 2, 1, 1.0, 64
    H1, H2 = widths
    rng = np.random.default_rng(31)
    scaler = StandardScaler().fit(rng.uniform(MC_LOW, MC_HIGH, (10000, S)))  # ddpg.py:186-189
    p = _noisy_params(O, S, A, H1, H2, seed=40)
    sess, actor, critic = _open(dd, O, S, A, H1, H2, scale, p, batch_max=B, scaler=scaler)
    rb = ReplayBuffer(4000, 1234)
    rows = _rows(rng, 3000, S, A, scale, np.float64, MC_LOW, MC_HIGH)
    rb.add_batch(*rows)
    assert rb.f64
    fl = FusedLearner(sess, rb, B)
    feed = lambda x: scaler.transform(x).astype(np.float32).astype(np.float64)
    L = O.Learner(S, A, H1, H2, scale, dtype=np.float64, params=p, init_blend=False)
    s_raw = rows[0][:B]
    # action selection at B = 1 and a batch (sb_actor_predict / GEMM path)
    for lo, hi in ((0, 1), (0, B)):
        mu = actor.predict(s_raw[lo:hi])
        assert rel(mu, L.actor_predict(feed(s_raw[lo:hi]))) < FWD_TOL, (lo, hi)
        mut = actor.predict_target(s_raw[lo:hi])
        assert rel(mut, L.actor_predict(feed(s_raw[lo:hi]), target=True)) < FWD_TOL
    q = critic.predict(s_raw, rows[1][:B])
    assert rel(q, L.critic_predict(feed(s_raw), rows[1][:B].astype(np.float64))) < FWD_TOL
    # one fused step from the float64 ring (device scaler)
    idx = np.array(random.Random(1234).sample(range(3000), B))
    qmax, loss = fl.step(stats=True)
    s, a, r, t, s2 = (x[idx] for x in rows)
    out = L.step(feed(s), a, r.astype(np.float32), t, feed(s2))
    assert abs(loss - float(out["loss"])) <= GRAD_TOL * abs(float(out["loss"]))
    assert abs(qmax - float(np.max(out["q"]))) <= 1e-5 * max(1.0, abs(float(np.max(out["q"]))))
    for which, net, keys in ((_lib.ACTOR, "actor", O.ACTOR_KEYS),
                             (_lib.CRITIC, "critic", O.CRITIC_KEYS)):
        for k, v in zip(keys, sess.get_params(which)):
            assert rel(v, L.state()[net][k].reshape(v.shape)) < GRAD_TOL, (net, k)
    # then the 1:1 methods on raw states: critic.train -> action_gradients -> actor.train
    s1, a1 = rows[0][100:100 + B], rows[1][100:100 + B]
    y = rng.standard_normal((B, 1)).astype(np.float32)
    qp, _, l1 = critic.train(s1, a1, y)
    q_ref, l_ref, _ = L.critic_train(feed(s1), a1.astype(np.float64), y.astype(np.float64))
    assert rel(qp, q_ref) < FWD_TOL and abs(float(l1) - l_ref) <= GRAD_TOL * abs(l_ref)
    a_out = actor.predict(s1)
    (da,) = critic.action_gradients(s1, a_out)
    da_ref = L.action_gradients(feed(s1), a_out.astype(np.float64))
    assert rel(da, da_ref) < GRAD_TOL
    actor.train(s1, da)
    L.actor_train(feed(s1), da.astype(np.float64))
    for which, net, keys in ((_lib.ACTOR, "actor", O.ACTOR_KEYS),
                             (_lib.CRITIC, "critic", O.CRITIC_KEYS)):
        for k, v in zip(keys, sess.get_params(which)):
            assert rel(v, L.state()[net][k].reshape(v.shape)) < GRAD_TOL, (net, k)
    # sample_batch returns the stored float64 rows exactly
    s_b, a_b, r_b, t_b, s2_b, pos = rb.sample_batch(16, return_indices=True)
    assert s_b.dtype == np.float64 and np.array_equal(s_b, rows[0][pos])
    assert np.array_equal(r_b, rows[2][pos]) and np.array_equal(s2_b, rows[4][pos])
    sess.close()


# ---------------------------------------------------------------- ragged shapes
@pytest.mark.parametrize("S,A,H1,H2,B,steps", [(17, 6, 400, 300, 600, 3),
                                               (64, 16, 1024, 1024, 4100, 2)])
def test_large_path_ragged_shapes(dd, O, S, A, H1, H2, B, steps):
    """The large-batch path on shapes that fill no tile.  (a) B = 600 (past
    the small path's 512, not a multiple of 64 or 128), S = 17 (thin_k's K
    padded to 24), A = 6, and the reference's 400 / 300 widths
    (parameters.py; 400 and 300 are not multiples of 128, and the concat
    2 x 400 not of 256): every GEMM has partial row and column tiles.  (b) the
    C3 widths at B = 4100, four rows past the headline batch: a partial last
    row tile on every batch-row GEMM and a ragged last K-split of every weight
    gradient.  Fused steps against the float64 oracle on the same sampled
    rows, with the fused-step bars of test_gpu_parity (fp32 restatement drift
    as the floor)."""
    from distributed_ddpg_amd import _lib
    from distributed_ddpg_amd.learner import FusedLearner, Profile
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    from test_gpu_parity import assert_steps_close
    scale = 2.0
    rng = np.random.default_rng(61)
    p = _noisy_params(O, S, A, H1, H2, seed=70)
    sess, actor, critic = _open(dd, O, S, A, H1, H2, scale, p, batch_max=B)
    n = max(3000, 2 * B)
    rb = ReplayBuffer(n + 1000, 1234)
    rows = _rows(rng, n, S, A, scale)
    rb.add_batch(*rows)
    fl = FusedLearner(sess, rb, B)
    L = O.Learner(S, A, H1, H2, scale, dtype=np.float64, params=p, init_blend=False)
    L32 = O.Learner(S, A, H1, H2, scale, dtype=np.float32, params=p, init_blend=False)
    prof = Profile(sess)
    prof.enable(True)
    ref_rng = random.Random(1234)
    for _ in range(steps):
        idx = np.array(ref_rng.sample(range(n), B))
        qmax, loss = fl.step(stats=True)
        s, a, r, t, s2 = (x[idx] for x in rows)
        out = L.step(s, a, r, t, s2)
        L32.step(s, a, r, t, s2)
        assert abs(loss - float(out["loss"])) <= GRAD_TOL * abs(float(out["loss"]))
        q_ref = float(np.max(out["q"]))
        assert abs(qmax - q_ref) <= FWD_TOL * max(1.0, abs(q_ref)) * 10
    keys = sorted(prof.read())
    prof.enable(False)
    assert not any(k.startswith("sb_") for k in keys), keys  # the large-batch path ran
    assert any(k.startswith("gemm_") for k in keys), keys
    for which, net, keys_ in ((_lib.ACTOR, "actor", O.ACTOR_KEYS),
                              (_lib.CRITIC, "critic", O.CRITIC_KEYS),
                              (_lib.ACTOR_TARGET, "actor_t", O.ACTOR_KEYS),
                              (_lib.CRITIC_TARGET, "critic_t", O.CRITIC_KEYS)):
        for k, v in zip(keys_, sess.get_params(which)):
            assert_steps_close(v, L.state()[net][k], L32.state()[net][k], (net, k))
    sess.close()


# ---------------------------------------------------------------- C3
def test_c3_gradients_and_adam_slots(dd, O):
    """B=4096, 1024/1024 (the headline shape): after one fused step the
    gradient buffers equal the oracle's gradients and the Adam slots are
    m = 0.1 g, v = 0.001 g^2 -- this pins every split-K slab reduction, the
    thin-K colsum bias gradients and the dX chains, not just parameter signs."""
    from distributed_ddpg_amd import _lib
    from distributed_ddpg_amd.learner import FusedLearner
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    S, A, H1, H2, scale, B = 64, 16, 1024, 1024, 1.0, 4096
    p = _noisy_params(O, S, A, H1, H2, seed=50)
    sess, actor, critic = _open(dd, O, S, A, H1, H2, scale, p, batch_max=B)
    rb = ReplayBuffer(20000, 77)
    rows = _rows(np.random.default_rng(9), 20000, S, A, scale)
    rb.add_batch(*rows)
    FusedLearner(sess, rb, B).step()
    idx = np.array(random.Random(77).sample(range(20000), B))
    L = O.Learner(S, A, H1, H2, scale, dtype=np.float64, params=p, init_blend=False)
    out = L.step(*(x[idx] for x in rows))
    for gw, mw, vw, ref, keys in (
            (_lib.CRITIC_GRAD, _lib.CRITIC_ADAM_M, _lib.CRITIC_ADAM_V, out["critic_grads"],
             O.CRITIC_KEYS),
            (_lib.ACTOR_GRAD, _lib.ACTOR_ADAM_M, _lib.ACTOR_ADAM_V, out["actor_grads"],
             O.ACTOR_KEYS)):
        for k, g, m, v in zip(keys, sess.get_params(gw), sess.get_params(mw), sess.get_params(vw)):
            r = ref[k].reshape(g.shape)
            assert rel(g, r) < GRAD_TOL, ("grad", k, rel(g, r))
            assert rel(m, 0.1 * r) < GRAD_TOL, ("m", k)
            assert rel(v, 0.001 * r * r) < 2 * GRAD_TOL, ("v", k)
    sess.close()


# ---------------------------------------------------------------- C4 (on one GPU)
def test_data_parallel_rank_slices_sum_to_global(dd, O, monkeypatch):
    """world=2, ranks 0 and 1 (no communicator, so each keeps its local
    gradient): each runs ddpg_learner_step on its slice [r*B/2, (r+1)*B/2) of
    the same global MT19937 draw with 1/B_global scaling.  Summed over ranks,
    the gradients and loss shares equal the world=1 global-batch step and the
    oracle.  critic_lr = 0 keeps the critic fixed (ApplyAdam with alpha = 0
    leaves it bit-unchanged), so the actor gradients, which use the updated
    critic, are comparable across world sizes too."""
    from distributed_ddpg_amd import _lib
    from distributed_ddpg_amd.learner import FusedLearner
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    monkeypatch.setenv("DDPG_SMALL", "0")
    S, A, H1, H2, scale, B = 4, 1, 128, 200, 3.0, 256
    p = _noisy_params(O, S, A, H1, H2, seed=60)
    rows = _rows(np.random.default_rng(61), 3000, S, A, scale)
    res = {}
    for world, rank in ((1, 0), (2, 0), (2, 1)):
        sess, actor, critic = _open(dd, O, S, A, H1, H2, scale, p, batch_max=B // world,
                                    rank=rank, world=world, critic_lr=0.0)
        rb = ReplayBuffer(5000, 1234)
        rb.add_batch(*rows)
        qmax, loss = FusedLearner(sess, rb, B).step(stats=True)
        res[(world, rank)] = (qmax, loss, sess.get_params(_lib.CRITIC_GRAD),
                              sess.get_params(_lib.ACTOR_GRAD), sess.get_params(_lib.CRITIC))
        sess.close()
    q1, l1, gc1, ga1, c1 = res[(1, 0)]
    q_a, l_a, gc_a, ga_a, c_a = res[(2, 0)]
    q_b, l_b, gc_b, ga_b, c_b = res[(2, 1)]
    for x, y in zip(c1, [p["critic"][k] for k in O.CRITIC_KEYS]):
        assert np.array_equal(x.ravel(), y.ravel())  # lr 0: critic unchanged
    idx = np.array(random.Random(1234).sample(range(3000), B))
    L = O.Learner(S, A, H1, H2, scale, critic_lr=0.0, dtype=np.float64, params=p,
                  init_blend=False)
    out = L.step(*(x[idx] for x in rows))
    assert abs((l_a + l_b) - l1) <= GRAD_TOL * abs(l1)
    assert abs(float(out["loss"]) - l1) <= GRAD_TOL * abs(l1)
    assert max(q_a, q_b) == pytest.approx(q1, rel=1e-5, abs=1e-6)
    for g1, ga, gb, ref, keys in ((gc1, gc_a, gc_b, out["critic_grads"], O.CRITIC_KEYS),
                                  (ga1, ga_a, ga_b, out["actor_grads"], O.ACTOR_KEYS)):
        for k, x1, xa, xb in zip(keys, g1, ga, gb):
            r = ref[k].reshape(x1.shape)
            assert rel(xa + xb, x1) < GRAD_TOL, ("sum vs world1", k)
            assert rel(xa + xb, r) < GRAD_TOL, ("sum vs oracle", k)
            assert rel(xa, r) > 1e-3 or np.max(np.abs(r)) == 0, ("rank slice is partial", k)


# ---------------------------------------------------------------- C5
BF16_FWD_TOL, BF16_DA_TOL, BF16_GRAD_NORM_TOL, BF16_PARAM_TOL = 2e-2, 5e-2, 3e-2, 2e-2
# Adam first-moment slot after the first step, m = (1 - beta1) g: max-rel bar
# (max |m - 0.1 g_ref| / max |0.1 g_ref|) against the float64 oracle gradient
BF16_M_MAXREL = 5e-2
# per-tensor max-rel gradient bar beside the norm-wise one: max |g - g_ref| /
# max |g_ref| over each tensor, so one bad row of a 2048-wide layer fails it
BF16_GRAD_MAXREL = 5e-2


def maxrel(x, r):
    x, r = np.asarray(x, np.float64), np.asarray(r, np.float64).reshape(np.shape(x))
    return float(np.max(np.abs(x - r)) / max(np.max(np.abs(r)), 1e-30))


def test_c5_bf16_full_dims(dd, O):
    """BASELINE configs[4]: S=376, A=17, 2048/2048, B=4096, bf16 GEMM operands
    with fp32 accumulation / master state.  A=17 sends Wa and the A-wide
    projections through the unaligned fp32 path.  Oracle in float64."""
    from distributed_ddpg_amd import _lib
    from distributed_ddpg_amd.learner import FusedLearner, Profile
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    S, A, H1, H2, scale, B = 376, 17, 2048, 2048, 1.0, 4096
    p = _noisy_params(O, S, A, H1, H2, seed=70, amp=0.02)
    sess, actor, critic = _open(dd, O, S, A, H1, H2, scale, p, batch_max=B, dtype="bf16")
    rng = np.random.default_rng(71)
    rows = _rows(rng, 6000, S, A, scale)
    s = rows[0][:512].astype(np.float64)
    mu = actor.predict(rows[0][:512])
    assert rel(mu, O.actor_forward(f64(p["actor"]), s, scale)[3]) < BF16_FWD_TOL
    q = critic.predict(rows[0][:512], rows[1][:512])
    assert rel(q, O.critic_forward(f64(p["critic"]), s, rows[1][:512].astype(np.float64))[3]) \
        < BF16_FWD_TOL
    (da,) = critic.action_gradients(rows[0][:512], mu)
    assert rel(da, O.critic_action_grads(f64(p["critic"]), s, mu.astype(np.float64))) \
        < BF16_DA_TOL
    rb = ReplayBuffer(8000, 1234)
    rb.add_batch(*rows)
    fl = FusedLearner(sess, rb, B)
    prof = Profile(sess)
    prof.enable(True)
    qmax, loss = fl.step(stats=True)
    keys = prof.read()
    prof.enable(False)
    assert any((k.startswith("gemm_s3_kernel") and "NP=1" in k) or
               (k.startswith("gemm_h") and "NP=1" in k) for k in keys), sorted(keys)
    idx = np.array(random.Random(1234).sample(range(6000), B))
    L = O.Learner(S, A, H1, H2, scale, dtype=np.float64, params=p, init_blend=False)
    out = L.step(*(x[idx] for x in rows))
    assert abs(loss - float(out["loss"])) <= 2e-2 * abs(float(out["loss"]))
    for gw, ref, keys_ in ((_lib.CRITIC_GRAD, out["critic_grads"], O.CRITIC_KEYS),
                           (_lib.ACTOR_GRAD, out["actor_grads"], O.ACTOR_KEYS)):
        for k, g in zip(keys_, sess.get_params(gw)):
            assert normrel(g, ref[k]) < BF16_GRAD_NORM_TOL, ("grad", k, normrel(g, ref[k]))
            assert maxrel(g, ref[k]) < BF16_GRAD_MAXREL, ("grad max-rel", k, maxrel(g, ref[k]))
    # Adam slots after the first step (fresh state): m = (1 - beta1) g and
    # v = (1 - beta2) g^2 of the GPU's own gradient, and m against the
    # oracle's gradient at the stated bf16 max-rel bar
    for gw, mw, vw, ref, keys_ in (
            (_lib.CRITIC_GRAD, _lib.CRITIC_ADAM_M, _lib.CRITIC_ADAM_V, out["critic_grads"],
             O.CRITIC_KEYS),
            (_lib.ACTOR_GRAD, _lib.ACTOR_ADAM_M, _lib.ACTOR_ADAM_V, out["actor_grads"],
             O.ACTOR_KEYS)):
        for k, g, m, v in zip(keys_, sess.get_params(gw), sess.get_params(mw), sess.get_params(vw)):
            g64, r = np.asarray(g, np.float64), 0.1 * np.asarray(ref[k], np.float64).reshape(g.shape)
            # TF ApplyAdam takes 1 - beta in fp32: 0.100000024, 0.00099998713
            c1 = float(np.float32(1) - np.float32(0.9))
            c2 = float(np.float32(1) - np.float32(0.999))
            assert np.max(np.abs(m - c1 * g64)) <= 1e-6 * np.max(np.abs(c1 * g64)) + 1e-30, ("m", k)
            assert np.max(np.abs(v - c2 * g64 * g64)) <= 1e-6 * np.max(c2 * g64 * g64) + 1e-30, \
                ("v", k)
            mr = np.max(np.abs(m - r)) / max(np.max(np.abs(r)), 1e-30)
            assert mr < BF16_M_MAXREL, ("m vs oracle", k, mr)
    # parameters after the step.  TF Adam's first step moves an element by
    # lr * g / (|g| + eps / sqrt(1 - beta2)) = lr * sign(g) for |g| >> 3e-7:
    # where the oracle's gradient is at least a tenth of its maximum (no bf16
    # sign flip possible there) the step must be -lr * sign(g_ref) to 1 % of lr;
    # elsewhere a sign flipped near zero costs at most two steps (2 lr), and the
    # weight matrices also meet the max-rel bar
    for which, net, names, lr, grads in ((_lib.ACTOR, "actor", O.ACTOR_KEYS, 1e-4,
                                          out["actor_grads"]),
                                         (_lib.CRITIC, "critic", O.CRITIC_KEYS, 1e-3,
                                          out["critic_grads"])):
        for k, v in zip(names, sess.get_params(which)):
            r = L.state()[net][k].reshape(v.shape)
            assert np.max(np.abs(v - r)) <= 2.02 * lr, (net, k, np.max(np.abs(v - r)))
            if k.startswith("W") and v.size >= 64 * 64:
                assert rel(v, r) < BF16_PARAM_TOL, (net, k)
            g = np.asarray(grads[k], np.float64).reshape(v.shape)
            big = np.abs(g) >= 0.1 * np.max(np.abs(g))
            th0 = np.asarray(p[net][k], np.float64).reshape(v.shape)
            step = np.asarray(v, np.float64) - th0
            tol = 0.01 * lr + 4 * np.spacing(np.abs(th0).astype(np.float32)).astype(np.float64)
            bad = big & (np.abs(step + lr * np.sign(g)) > tol)
            assert not bad.any(), (net, k, int(bad.sum()), int(big.sum()))
    sess.close()


def test_bf16_ragged_shapes(dd, O):
    """The bf16 configuration on shapes that fill no tile: S = 100 (first
    layers on the GEMMs, K not a multiple of the 64-deep step), A = 7, widths
    600 / 520 (not multiples of 128 or 256), B = 1000 (not a multiple of the
    256-row tile).  One fused step against the float64 oracle at the stated
    bf16 bars of test_c5_bf16_full_dims: loss, gradients norm-wise and max-rel
    per tensor, every parameter within two Adam steps."""
    from distributed_ddpg_amd import _lib
    from distributed_ddpg_amd.learner import FusedLearner
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    S, A, H1, H2, scale, B = 100, 7, 600, 520, 1.0, 1000
    p = _noisy_params(O, S, A, H1, H2, seed=80, amp=0.02)
    sess, actor, critic = _open(dd, O, S, A, H1, H2, scale, p, batch_max=B, dtype="bf16")
    rng = np.random.default_rng(81)
    rows = _rows(rng, 3000, S, A, scale)
    rb = ReplayBuffer(4000, 1234)
    rb.add_batch(*rows)
    fl = FusedLearner(sess, rb, B)
    qmax, loss = fl.step(stats=True)
    idx = np.array(random.Random(1234).sample(range(3000), B))
    L = O.Learner(S, A, H1, H2, scale, dtype=np.float64, params=p, init_blend=False)
    out = L.step(*(x[idx] for x in rows))
    assert abs(loss - float(out["loss"])) <= 2e-2 * abs(float(out["loss"]))
    for gw, ref, keys_ in ((_lib.CRITIC_GRAD, out["critic_grads"], O.CRITIC_KEYS),
                           (_lib.ACTOR_GRAD, out["actor_grads"], O.ACTOR_KEYS)):
        for k, g in zip(keys_, sess.get_params(gw)):
            assert normrel(g, ref[k]) < BF16_GRAD_NORM_TOL, ("grad", k, normrel(g, ref[k]))
            assert maxrel(g, ref[k]) < BF16_GRAD_MAXREL, ("grad max-rel", k, maxrel(g, ref[k]))
    for which, net, names, lr in ((_lib.ACTOR, "actor", O.ACTOR_KEYS, 1e-4),
                                  (_lib.CRITIC, "critic", O.CRITIC_KEYS, 1e-3)):
        for k, v in zip(names, sess.get_params(which)):
            r = L.state()[net][k].reshape(v.shape)
            assert np.max(np.abs(v - r)) <= 2.02 * lr, (net, k, np.max(np.abs(v - r)))
    sess.close()
