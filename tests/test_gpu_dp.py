"""GPU tests of the per-rank data-parallel path on one GPU:

  * the small-M plan (in-launch K split of the forward / dX twin GEMMs,
    ksplit_combine) at a strong-scaling per-rank batch of the headline shape
    (C3 widths, B = 512: rank 0 of 8) against the oracle, graph vs eager bitwise;
  * DDPG_KCOMB=0 (no in-launch split) against the oracle;
  * the proxy communicator (ddpg_comm_init_proxy): one GPU runs rank 0's share
    of an 8-rank step -- its slice of the global draw, every RCCL call site --
    checked against the oracle on that slice; the step graph with the RCCL
    calls captured equals the eager step bitwise;
  * the comm-stream ordering (DDPG_TEST_CS_SPIN): a kernel on the comm stream
    that waits, then doubles the exchanged gradient ranges; Adam must see the
    doubled values (profiling off, graph and eager, one and three streams).

Bars as tests/test_gpu_configs.py: gradients / Adam slots 1e-4 (fp32).
"""
import random

import numpy as np
import pytest

from test_gpu_configs import _noisy_params, _open, _rows
from test_gpu_parity import CONFIGS, GRAD_TOL, _fill, _params, _session, rel

pytestmark = pytest.mark.gpu

ENV = ("DDPG_KCOMB", "DDPG_KCOMB_BLOCKS", "DDPG_GRAPH", "DDPG_GRAPH_COMM", "DDPG_GRAPH_AUTO",
       "DDPG_PAR", "DDPG_GEMM_M16",
       "DDPG_TEST_CS_SPIN", "DDPG_SMALL")


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


@pytest.fixture
def clean_env(monkeypatch):
    for k in ENV:
        monkeypatch.delenv(k, raising=False)
    return monkeypatch


def _state(sess):
    from distributed_ddpg_amd import _lib
    return [sess.get_params(w) for w in (_lib.ACTOR, _lib.CRITIC, _lib.ACTOR_TARGET,
                                         _lib.CRITIC_TARGET, _lib.ACTOR_ADAM_M, _lib.ACTOR_ADAM_V,
                                         _lib.CRITIC_ADAM_M, _lib.CRITIC_ADAM_V, _lib.ACTOR_GRAD,
                                         _lib.CRITIC_GRAD)]


def _same(a, b):
    for x, y in zip(a, b):
        for u, v in zip(x, y):
            assert np.array_equal(u, v)


C3 = (64, 16, 1024, 1024, 1.0)


def _c3_run(dd, O, p, rows, B, Bg, world=1, proxy=False, profile=False, critic_lr=1e-3,
            seed=77):
    from distributed_ddpg_amd import _lib
    from distributed_ddpg_amd.learner import FusedLearner, Profile
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    S, A, H1, H2, scale = C3
    sess, actor, critic = _open(dd, O, S, A, H1, H2, scale, p, batch_max=B, rank=0, world=world,
                                critic_lr=critic_lr)
    if proxy:
        _lib.check(_lib.lib.ddpg_comm_init_proxy(sess.ctx), sess.ctx)
    rb = ReplayBuffer(len(rows[0]) + 1000, seed)
    rb.add_batch(*rows)
    fl = FusedLearner(sess, rb, Bg)
    prof = Profile(sess)
    if profile:
        prof.enable(True)
    st = fl.step(stats=True)
    keys = sorted(prof.read()) if profile else []
    if profile:
        prof.enable(False)
    out = _state(sess), st, keys, fl.step_counts()
    sess.close()
    return out


def test_small_m_plan_c3_b512(dd, O, clean_env):
    """C3 widths at B = 512 (the per-rank batch of an 8-GPU strong-scaling
    run): the forward and dX twin GEMMs (32 / 32-64 output tiles) split K
    and combine in-launch.  One fused step: every gradient and the Adam slots
    at 1e-4 of the float64 oracle; the graph replay and the profiled eager
    step are bitwise equal (the combine sums the splits in a fixed order)."""
    S, A, H1, H2, scale = C3
    B = 512
    p = _noisy_params(O, S, A, H1, H2, seed=50)
    rows = _rows(np.random.default_rng(9), 6000, S, A, scale)
    g_state, g_st, _, g_cnt = _c3_run(dd, O, p, rows, B, B)
    e_state, e_st, keys, e_cnt = _c3_run(dd, O, p, rows, B, B, profile=True)
    assert g_cnt == (1, 0, False) and e_cnt == (0, 1, False), (g_cnt, e_cnt)
    assert any(k.startswith("gemm_h3_kernel<RK,KR") and k.endswith("/kc") for k in keys), keys
    assert any(k.startswith("gemm_h3_kernel<RK,RK") and k.endswith("/kc") for k in keys), keys
    _same(g_state, e_state)
    assert g_st == e_st
    idx = np.array(random.Random(77).sample(range(6000), B))
    L = O.Learner(S, A, H1, H2, scale, dtype=np.float64, params=p, init_blend=False)
    out = L.step(*(x[idx] for x in rows))
    assert abs(g_st[1] - float(out["loss"])) <= GRAD_TOL * abs(float(out["loss"]))
    for gi, mi, vi, ref, keys_ in ((9, 6, 7, out["critic_grads"], O.CRITIC_KEYS),
                                   (8, 4, 5, out["actor_grads"], O.ACTOR_KEYS)):
        for k, g, m, v in zip(keys_, g_state[gi], g_state[mi], g_state[vi]):
            r = ref[k].reshape(g.shape)
            assert rel(g, r) < GRAD_TOL, ("grad", k, rel(g, r))
            assert rel(m, 0.1 * r) < GRAD_TOL, ("m", k)
            assert rel(v, 0.001 * r * r) < 2 * GRAD_TOL, ("v", k)


def test_kcomb_off_matches_oracle(dd, O, clean_env):
    """DDPG_KCOMB=0: the same small-M GEMMs unsplit (32 blocks each) --
    no "/kc" launches, and the 1e-4 gradient bars hold."""
    S, A, H1, H2, scale = C3
    B = 512
    clean_env.setenv("DDPG_KCOMB", "0")
    p = _noisy_params(O, S, A, H1, H2, seed=51)
    rows = _rows(np.random.default_rng(10), 6000, S, A, scale)
    state, st, keys, _ = _c3_run(dd, O, p, rows, B, B, profile=True)
    assert not any(k.endswith("/kc") for k in keys), keys
    idx = np.array(random.Random(77).sample(range(6000), B))
    L = O.Learner(S, A, H1, H2, scale, dtype=np.float64, params=p, init_blend=False)
    out = L.step(*(x[idx] for x in rows))
    for gi, ref, keys_ in ((9, out["critic_grads"], O.CRITIC_KEYS),
                           (8, out["actor_grads"], O.ACTOR_KEYS)):
        for k, g in zip(keys_, state[gi]):
            assert rel(g, ref[k].reshape(g.shape)) < GRAD_TOL, ("grad", k)


def test_proxy_rank0_of_8_c3(dd, O, clean_env):
    """bench.py --per-rank-of 8 (strong): world = 8, rank 0, per-rank batch
    512 of a global 4096 draw, proxy communicator.  The step samples the
    global batch, gathers rank 0's slice and runs every RCCL call site (a
    1-rank identity).  critic_lr = 0 keeps the critic fixed, so: the critic
    gradient = the oracle's mean over the slice x 512/4096 (the loss is scaled
    by 1/B_global), the actor gradient = the oracle's batch sum over the slice,
    the loss share = the slice loss / 8.  The graph with the RCCL calls
    captured and the eager step (DDPG_GRAPH_COMM=0) are bitwise equal."""
    S, A, H1, H2, scale = C3
    B, Bg, world = 512, 4096, 8
    p = _noisy_params(O, S, A, H1, H2, seed=52)
    rows = _rows(np.random.default_rng(11), 9000, S, A, scale)
    g_state, g_st, _, g_cnt = _c3_run(dd, O, p, rows, B, Bg, world=world, proxy=True,
                                      critic_lr=0.0)
    # the RCCL calls were captured with the step (not a silent eager fallback)
    assert g_cnt == (1, 0, False), g_cnt
    clean_env.setenv("DDPG_GRAPH_COMM", "0")
    e_state, e_st, keys, e_cnt = _c3_run(dd, O, p, rows, B, Bg, world=world, proxy=True,
                                         critic_lr=0.0, profile=True)
    assert e_cnt == (0, 1, False), e_cnt
    assert "rccl_allreduce" in keys and "rccl_stats" in keys, keys
    assert any(k.startswith("xwin|") for k in keys), keys
    # the weight gradients' K splits combined in-launch (no slab reduction in
    # front of their all-reduce)
    assert any(k.startswith("gemm_h3m_kernel<KR,KR") and k.endswith("/kc") for k in keys), keys
    _same(g_state, e_state)
    assert g_st == e_st
    idx = np.array(random.Random(77).sample(range(9000), Bg))[:B]
    L = O.Learner(S, A, H1, H2, scale, critic_lr=0.0, dtype=np.float64, params=p,
                  init_blend=False)
    out = L.step(*(x[idx] for x in rows))
    assert abs(g_st[1] - float(out["loss"]) / world) <= GRAD_TOL * abs(float(out["loss"]) / world)
    assert abs(g_st[0] - float(np.max(out["q"]))) <= 1e-5 * max(1.0, abs(float(np.max(out["q"]))))
    for gi, ref, keys_, f in ((9, out["critic_grads"], O.CRITIC_KEYS, 1.0 / world),
                              (8, out["actor_grads"], O.ACTOR_KEYS, 1.0)):
        for k, g in zip(keys_, g_state[gi]):
            assert rel(g, f * ref[k].reshape(g.shape)) < GRAD_TOL, ("grad", k)


def _wide_comm(dd, O, name, p, spin=0, comm=True):
    from distributed_ddpg_amd.learner import FusedLearner, init_comm
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    S, A, H1, H2, scale, B, _ = CONFIGS[name]
    sess, actor, critic = _session(dd, O, name, p, batch_max=1024)
    if comm:
        init_comm(sess, 0, 1, single=True)
    rb = ReplayBuffer(5000, 1234)
    _fill(rb, S, A, 3000, scale, seed=2)
    fl = FusedLearner(sess, rb, 1024)
    st = fl.step(stats=True)
    out = _state(sess), st, fl.step_counts()
    sess.close()
    return out


@pytest.mark.parametrize("graph_comm", ["1", "0"])
def test_comm_graph_matches_no_comm(dd, O, clean_env, graph_comm):
    """A 1-rank communicator's exchange is an identity: with the step graph
    capturing the RCCL calls (default) and eagerly (DDPG_GRAPH_COMM=0), one
    fused step equals the communicator-less step bitwise (profiling off)."""
    p, _ = _params(O, "wide")
    ref = _wide_comm(dd, O, "wide", p, comm=False)
    clean_env.setenv("DDPG_GRAPH_COMM", graph_comm)
    got = _wide_comm(dd, O, "wide", p)
    # graph_comm=1: the step was replayed from a graph holding the RCCL calls
    # (a failed capture would fall back to eager and pass the equality trivially)
    assert got[2] == ((1, 0, False) if graph_comm == "1" else (0, 1, False)), got[2]
    _same(got[0], ref[0])
    assert got[1] == ref[1]


@pytest.mark.parametrize("par,graph_comm", [("0", "1"), ("1", "1"), ("0", "0"), ("1", "0")])
def test_comm_stream_ordering_spin(dd, O, clean_env, par, graph_comm):
    """DDPG_TEST_CS_SPIN=300: on the comm stream, ahead of each collective
    group, a kernel waits 300 us and then doubles the ranges the group
    exchanges.  If Adam (or the slab reduction writing the tail ranges) were
    not ordered behind the comm stream it would read undoubled gradients.
    Checks, profiling off: the critic gradient buffer is exactly 2x the
    no-spin run's and its Adam slots exactly 2x / 4x (fresh slots: m =
    (1 - b1) g, v = (1 - b2) g^2 scale exactly by powers of two); for both
    networks m == (1 - b1) G and v == (1 - b2) G^2 of the final buffer G, bitwise
    with TF's formula (Adam consumed the doubled values)."""
    p, _ = _params(O, "wide")
    clean_env.setenv("DDPG_PAR", par)
    clean_env.setenv("DDPG_GRAPH_COMM", graph_comm)
    ref = _wide_comm(dd, O, "wide", p)
    clean_env.setenv("DDPG_TEST_CS_SPIN", "300")
    got = _wide_comm(dd, O, "wide", p)
    assert got[2] == ((1, 0, False) if graph_comm == "1" else (0, 1, False)), got[2]
    state, ref_state = got[0], ref[0]
    for g, g0 in zip(state[9], ref_state[9]):           # critic gradient
        assert np.array_equal(g, 2 * g0)
    for m, m0 in zip(state[6], ref_state[6]):
        assert np.array_equal(m, 2 * m0)
    for v, v0 in zip(state[7], ref_state[7]):
        assert np.array_equal(v, 4 * v0)
    one = np.float32(1)
    c1, c2 = one - np.float32(0.9), one - np.float32(0.999)
    for gi, mi, vi in ((9, 6, 7), (8, 4, 5)):
        for g, m, v in zip(state[gi], state[mi], state[vi]):
            g = g.astype(np.float32)
            assert np.array_equal(m, (g - np.float32(0)) * c1)
            assert np.array_equal(v, (g * g - np.float32(0)) * c2)


def test_ksplit_combine_deterministic_c5_b1024(dd, O, clean_env):
    """The in-launch K split at a second shape: the bf16 configuration at C5
    widths (S = 376, A = 17, 2048 / 2048) with B = 1024 (rank 0 of a 4-rank
    strong run), where the forward and dX gemm_h16i launches split K and
    combine in-launch.  Two fresh sessions run the same three fused steps --
    every gradient, Adam slot and parameter is bitwise equal between them
    (the combine adds the splits in split order, whatever order they land
    in), and the split launches really ran ("/kc" keys)."""
    from distributed_ddpg_amd.learner import FusedLearner, Profile
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    S, A, H1, H2, scale = 376, 17, 2048, 2048, 1.0
    B = 1024
    p = _noisy_params(O, S, A, H1, H2, seed=53)
    rows = _rows(np.random.default_rng(12), 3000, S, A, scale)
    runs = []
    for rep in range(2):
        sess, actor, critic = _open(dd, O, S, A, H1, H2, scale, p, batch_max=B, dtype="bf16")
        rb = ReplayBuffer(4000, 99)
        rb.add_batch(*rows)
        fl = FusedLearner(sess, rb, B)
        prof = Profile(sess)
        if rep == 1:
            prof.enable(True)
        st = [fl.step(stats=True) for _ in range(3)]
        keys = sorted(prof.read()) if rep == 1 else []
        if rep == 1:
            prof.enable(False)
        runs.append((_state(sess), st, keys))
        sess.close()
    keys = runs[1][2]
    assert any(k.startswith("gemm_h16i_kernel<RK,KR") and k.endswith("/kc") for k in keys), keys
    assert any(k.startswith("gemm_h16i_kernel<RK,RK") and k.endswith("/kc") for k in keys), keys
    assert runs[0][1] == runs[1][1]
    _same(runs[0][0], runs[1][0])


IP = (4, 1, 128, 200, 3.0)   # InvertedPendulum widths (networks.py:54-55,151-156)


def _ip_run(dd, O, p, rows, B, Bg, world=1, comm=None, profile=False, critic_lr=1e-3, steps=1):
    from distributed_ddpg_amd import _lib
    from distributed_ddpg_amd.learner import FusedLearner, Profile, init_comm
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    S, A, H1, H2, scale = IP
    sess, actor, critic = _open(dd, O, S, A, H1, H2, scale, p, batch_max=B, world=world,
                                critic_lr=critic_lr)
    if comm == "proxy":
        _lib.check(_lib.lib.ddpg_comm_init_proxy(sess.ctx), sess.ctx)
    elif comm == "single":
        init_comm(sess, 0, 1, single=True)
    rb = ReplayBuffer(len(rows[0]) + 1000, 77)
    rb.add_batch(*rows)
    fl = FusedLearner(sess, rb, Bg)
    prof = Profile(sess)
    if profile:
        prof.enable(True)
    st = [fl.step(stats=True) for _ in range(steps)]
    keys = sorted(prof.read()) if profile else []
    if profile:
        prof.enable(False)
    out = _state(sess), st, keys, fl.step_counts(), fl.read_stats()
    sess.close()
    return out


@pytest.mark.parametrize("graph_comm", ["1", "0"])
def test_small_path_communicator_matches_no_comm(dd, O, clean_env, graph_comm):
    """Data parallelism at the reference's own shape (InvertedPendulum widths,
    B = 256 per worker, parameters.py:11,32-34) stays on the small-batch
    kernels: with a communicator each network's gradient / Adam kernel runs
    as two launches around the RCCL sum of its gradient range.  Through a
    1-rank communicator (an identity exchange) three fused steps equal the
    communicator-less step bitwise -- state, per-step stats and running sums
    -- replayed from a graph holding the RCCL calls or launched eagerly
    (DDPG_GRAPH_AUTO=1: the synchronised steps replay the graph; the small
    path's default issues every step eagerly)."""
    S, A, H1, H2, scale = IP
    clean_env.setenv("DDPG_GRAPH_AUTO", "1")
    p = _noisy_params(O, S, A, H1, H2, seed=60)
    rows = _rows(np.random.default_rng(20), 3000, S, A, scale)
    ref = _ip_run(dd, O, p, rows, 256, 256, steps=3)
    clean_env.setenv("DDPG_GRAPH_COMM", graph_comm)
    got = _ip_run(dd, O, p, rows, 256, 256, comm="single", steps=3)
    assert got[3] == ((3, 0, False) if graph_comm == "1" else (0, 3, False)), got[3]
    _same(got[0], ref[0])
    assert got[1] == ref[1]
    assert got[4] == ref[4]
    _, _, keys, _, _ = _ip_run(dd, O, p, rows, 256, 256, comm="single", profile=True)
    for k in ("sb_phase1", "sb_phase3", "sb_wgrad_adam", "sb_adam", "rccl_allreduce", "rccl_stats"):
        assert k in keys, (k, keys)
    assert not any(k.startswith("gemm_") for k in keys), keys


def test_small_path_proxy_rank0_of_8(dd, O, clean_env):
    """Rank 0 of an 8-rank data-parallel step at B = 256 per rank (global
    2048) on the small-batch kernels, proxy communicator: with critic_lr = 0
    the critic gradient = the oracle's mean over rank 0's slice x 256/2048,
    the actor gradient = the oracle's batch sum over the slice, the loss
    share = the slice loss / 8 (1e-4)."""
    S, A, H1, H2, scale = IP
    B, Bg, world = 256, 2048, 8
    p = _noisy_params(O, S, A, H1, H2, seed=61)
    rows = _rows(np.random.default_rng(21), 5000, S, A, scale)
    state, st, keys, cnt, _ = _ip_run(dd, O, p, rows, B, Bg, world=world, comm="proxy",
                                      critic_lr=0.0, profile=True)
    assert "sb_adam" in keys and "rccl_allreduce" in keys, keys
    idx = np.array(random.Random(77).sample(range(5000), Bg))[:B]
    L = O.Learner(S, A, H1, H2, scale, critic_lr=0.0, dtype=np.float64, params=p,
                  init_blend=False)
    out = L.step(*(x[idx] for x in rows))
    q_max, loss = st[0]
    assert abs(loss - float(out["loss"]) / world) <= GRAD_TOL * abs(float(out["loss"]) / world)
    assert abs(q_max - float(np.max(out["q"]))) <= 1e-5 * max(1.0, abs(float(np.max(out["q"]))))
    for gi, ref, keys_, f in ((9, out["critic_grads"], O.CRITIC_KEYS, 1.0 / world),
                              (8, out["actor_grads"], O.ACTOR_KEYS, 1.0)):
        for k, g in zip(keys_, state[gi]):
            assert rel(g, f * ref[k].reshape(g.shape)) < GRAD_TOL, ("grad", k)


def test_proxy_rank0_of_8_c5_bf16_exchange(dd, O, clean_env):
    """The bf16 configuration at C5 dimensions (S = 376, A = 17, 2048 / 2048)
    exchanges its gradients as an fp32 reduce-scatter, one bf16 rounding of
    each rank's summed slice, a bf16 all-gather, widened back for Adam (6
    instead of 8 B per element on the links; at N = 1 one rounding of the
    rank's fp32 gradient).  Rank 0 of 8 at 512 rows per rank through the proxy
    communicator, critic_lr = 0: the critic gradient = the oracle's slice
    mean x 512/4096, the actor gradient = the slice sum, at the stated bf16
    bars (norm-wise and per-tensor max-rel); the exchanged buffers hold
    bf16-representable values; the step was a graph replay."""
    from test_gpu_configs import BF16_GRAD_MAXREL, BF16_GRAD_NORM_TOL, maxrel
    from test_gpu_parity import normrel
    from distributed_ddpg_amd import _lib
    from distributed_ddpg_amd.learner import FusedLearner
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    S, A, H1, H2, scale = 376, 17, 2048, 2048, 1.0
    B, Bg, world = 512, 4096, 8
    p = _noisy_params(O, S, A, H1, H2, seed=62, amp=0.02)
    rows = _rows(np.random.default_rng(22), 6000, S, A, scale)
    sess, actor, critic = _open(dd, O, S, A, H1, H2, scale, p, batch_max=B, world=world,
                                dtype="bf16", critic_lr=0.0)
    _lib.check(_lib.lib.ddpg_comm_init_proxy(sess.ctx), sess.ctx)
    rb = ReplayBuffer(8000, 77)
    rb.add_batch(*rows)
    fl = FusedLearner(sess, rb, Bg)
    q_max, loss = fl.step(stats=True)
    assert fl.step_counts() == (1, 0, False)
    state = _state(sess)
    sess.close()
    idx = np.array(random.Random(77).sample(range(6000), Bg))[:B]
    L = O.Learner(S, A, H1, H2, scale, critic_lr=0.0, dtype=np.float64, params=p,
                  init_blend=False)
    out = L.step(*(x[idx] for x in rows))
    assert abs(loss - float(out["loss"]) / world) <= 2e-2 * abs(float(out["loss"]) / world)
    for gi, ref, keys_, f in ((9, out["critic_grads"], O.CRITIC_KEYS, 1.0 / world),
                              (8, out["actor_grads"], O.ACTOR_KEYS, 1.0)):
        for k, g in zip(keys_, state[gi]):
            r = f * np.asarray(ref[k], np.float64).reshape(g.shape)
            assert normrel(g, r) < BF16_GRAD_NORM_TOL, ("grad", k, normrel(g, r))
            assert maxrel(g, r) < BF16_GRAD_MAXREL, ("grad max-rel", k, maxrel(g, r))
            g32 = np.asarray(g, np.float32)
            # exchanged as bf16: the low 16 bits of every fp32 value are zero
            assert np.all((g32.view(np.uint32) & 0xFFFF) == 0), k


def _bf16_rne(x):
    """fp32 -> bf16 (round to nearest even) -> fp32, as the exchange's
    f32_to_bf16_kernel rounds."""
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32)


def _ring_rs_fp32(parts):
    """Ring reduce-scatter in fp32: slice j's owner ends the ring, so its sum
    starts at rank j + 1 and adds the ranks in ring order (each partial sum
    rounded to fp32)."""
    n = len(parts)
    flat = [np.asarray(p, np.float32).ravel() for p in parts]
    m = flat[0].size - flat[0].size % n
    ch = m // n
    out = np.empty(flat[0].size, np.float32)
    for j in range(n):
        sl = slice(j * ch, (j + 1) * ch)
        acc = flat[(j + 1) % n][sl].copy()
        for k in range(2, n + 1):
            acc = (acc + flat[(j + k) % n][sl]).astype(np.float32)
        out[sl] = _bf16_rne(acc)
    tail = slice(m, flat[0].size)   # all-reduced in fp32
    acc = flat[0][tail].copy()
    for k in range(1, n):
        acc = (acc + flat[k][tail]).astype(np.float32)
    out[tail] = acc
    return out, m


def _ring_ar_bf16(parts):
    """The round-5 exchange for comparison: every rank's gradient rounded to
    bf16, then a bf16 ring sum (each hop's partial rounded to bf16)."""
    n = len(parts)
    acc = _bf16_rne(parts[0])
    for k in range(1, n):
        acc = _bf16_rne(acc.astype(np.float32) + _bf16_rne(parts[k]))
    return acc


def test_bf16_exchange_fp32_accumulation_8_ranks(dd, O, clean_env):
    """SURVEY §8(e) step 3, "bf16 with fp32 accumulation", at C5 dimensions
    and N = 8: the eight ranks' fp32 gradients are computed on the GPU (eight
    world = 8 contexts, no communicator, 512 rows each of the same global
    draw of 4096, critic_lr = 0); the exchange the build issues (csrc/dp.hip:
    fp32 ring reduce-scatter, one bf16 rounding of each slice, bf16
    all-gather; the n % 8 tail all-reduced in fp32) is emulated on the host
    with the same per-element arithmetic (the slices follow the concatenated
    tensors here, the flat buffer's padded ranges in the product).  Its result: every element within one bf16 rounding (2^-8
    relative) of the fp32 sum, the global-batch oracle gradient at the stated
    bf16 bars, and no worse than the round-5 bf16 ring sum (per-hop rounding)
    norm-wise.  The RCCL calls themselves run at N = 1 through the proxy
    (test_proxy_rank0_of_8_c5_bf16_exchange)."""
    from test_gpu_configs import BF16_GRAD_MAXREL, BF16_GRAD_NORM_TOL, maxrel
    from test_gpu_parity import normrel
    from distributed_ddpg_amd import _lib
    from distributed_ddpg_amd.learner import FusedLearner
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    S, A, H1, H2, scale = 376, 17, 2048, 2048, 1.0
    world, Bg = 8, 4096
    B = Bg // world
    p = _noisy_params(O, S, A, H1, H2, seed=63, amp=0.02)
    rows = _rows(np.random.default_rng(23), 6000, S, A, scale)
    grads = {"critic": [], "actor": []}
    for rank in range(world):
        sess, actor, critic = _open(dd, O, S, A, H1, H2, scale, p, batch_max=B, rank=rank,
                                    world=world, dtype="bf16", critic_lr=0.0)
        rb = ReplayBuffer(8000, 78)
        rb.add_batch(*rows)
        FusedLearner(sess, rb, Bg).step()
        grads["critic"].append(np.concatenate([g.ravel() for g in
                                               sess.get_params(_lib.CRITIC_GRAD)]))
        grads["actor"].append(np.concatenate([g.ravel() for g in
                                              sess.get_params(_lib.ACTOR_GRAD)]))
        sess.close()
    idx = np.array(random.Random(78).sample(range(6000), Bg))
    L = O.Learner(S, A, H1, H2, scale, critic_lr=0.0, dtype=np.float64, params=p,
                  init_blend=False)
    out = L.step(*(x[idx] for x in rows))
    for net, ref, keys in (("critic", out["critic_grads"], O.CRITIC_KEYS),
                           ("actor", out["actor_grads"], O.ACTOR_KEYS)):
        parts = grads[net]
        new, m = _ring_rs_fp32(parts)
        old = _ring_ar_bf16(parts)
        st = np.stack(parts).astype(np.float64)
        s32, sabs = st.sum(axis=0), np.abs(st).sum(axis=0)
        assert m > 0.99 * new.size
        # one bf16 rounding of the sum (2^-9 |x|) + the fp32 ring's partial sums
        # (<= (N - 1) 2^-24 sum |parts|, what cancellation leaves relative)
        assert np.all(np.abs(new - s32) <= 2.0 ** -8 * np.abs(s32) + world * 2.0 ** -24 * sabs
                      + 1e-30), net
        r = np.concatenate([np.asarray(ref[k], np.float64).ravel() for k in keys])
        e_new, e_old = normrel(new, r), normrel(old, r)
        assert e_new <= e_old * 1.0001 + 1e-7, (net, e_new, e_old)
        off = 0
        for k in keys:
            n = np.asarray(ref[k]).size
            g, rk = new[off:off + n], r[off:off + n]
            off += n
            assert normrel(g, rk) < BF16_GRAD_NORM_TOL, (net, k, normrel(g, rk))
            assert maxrel(g, rk) < BF16_GRAD_MAXREL, (net, k, maxrel(g, rk))
