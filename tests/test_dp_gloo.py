"""Synchronous data parallelism, world_size 2 on CPU (gloo).

The HIP path shards a globally drawn batch across ranks and sums gradients
with RCCL (DESIGN.md "Multi-GPU").  These tests pin that decomposition with
the oracle and real torch.distributed collectives:
  * every rank draws the SAME global positions (same MT19937 stream) and takes
    rows [r*B/N, (r+1)*B/N); the union is the 1-rank batch;
  * critic: local dQ = -(2(y-q))/B_global, local grads SUMMED == global mean
    grads; actor: local batch-sum grads SUMMED == global sum;
  * replicated TF-Adam on identical summed grads keeps ranks bit-identical
    and equal to the single-rank global-batch update;
  * the 128-byte RCCL unique id reaches every rank intact (init_comm's
    broadcast over the gloo group).
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(rank, world, port):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _problem(S=5, A=2, H1=12, H2=16, B=32, seed=0):
    from oracle import ddpg_oracle as O
    a, c = O.init_params(S, A, H1, H2, seed=seed, dtype=np.float64)
    rng = np.random.default_rng(seed + 1)
    for d in (a, c):
        for k in d:
            d[k] = d[k] + rng.standard_normal(d[k].shape) * 0.2
    s = rng.standard_normal((B, S))
    act = rng.standard_normal((B, A))
    y = rng.standard_normal((B, 1))
    dqa = rng.standard_normal((B, A))
    return O, a, c, s, act, y, dqa


def _dp_worker(rank, world, port, q):
    import torch
    _setup(rank, world, port)
    O, a, c, s, act, y, dqa = _problem()
    B = s.shape[0]
    lo, hi = rank * B // world, (rank + 1) * B // world
    # critic: local rows, global 1/B scaling (critic_loss_kernel's inv_b)
    qv = O.critic_forward(c, s[lo:hi], act[lo:hi])[3]
    dq = -((1.0 / B) * (2.0 * (y[lo:hi] - qv)))
    gc, _, _ = O.critic_grads(c, s[lo:hi], act[lo:hi], dq)
    ga = O.actor_grads(a, s[lo:hi], dqa[lo:hi], 1.5)
    flat = np.concatenate([gc[k].ravel() for k in O.CRITIC_KEYS] +
                          [ga[k].ravel() for k in O.ACTOR_KEYS])
    t = torch.from_numpy(flat.copy())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    # replicated Adam on the summed gradients
    opt_c = O.TFAdam(O.critic_shapes(5, 2, 12, 16), 1e-3, np.float64)
    opt_a = O.TFAdam(O.actor_shapes(5, 2, 12, 16), 1e-4, np.float64)
    g = t.numpy()
    o = 0
    gcs, gas = {}, {}
    for k in O.CRITIC_KEYS:
        n = c[k].size
        gcs[k] = g[o:o + n].reshape(c[k].shape)
        o += n
    for k in O.ACTOR_KEYS:
        n = a[k].size
        gas[k] = g[o:o + n].reshape(a[k].shape)
        o += n
    opt_c.apply(c, gcs)
    opt_a.apply(a, gas)
    q.put((rank, g, {k: c[k] for k in c}, {k: a[k] for k in a}))
    dist.destroy_process_group()


def test_dp_gradient_decomposition_matches_global_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-rank reference on the global batch
    O, a, c, s, act, y, dqa = _problem()
    q1 = O.critic_forward(c, s, act)[3]
    _, dq = O.mse_loss_and_grad(y, q1)
    gc, _, _ = O.critic_grads(c, s, act, dq)
    ga = O.actor_grads(a, s, dqa, 1.5)
    ref = np.concatenate([gc[k].ravel() for k in O.CRITIC_KEYS] +
                         [ga[k].ravel() for k in O.ACTOR_KEYS])
    for rank, g, cc, aa in res:
        np.testing.assert_allclose(g, ref, rtol=1e-12, atol=1e-14)
    # ranks stay bit-identical after replicated Adam
    for k in res[0][2]:
        assert np.array_equal(res[0][2][k], res[1][2][k])
    for k in res[0][3]:
        assert np.array_equal(res[0][3][k], res[1][3][k])


def _id_worker(rank, world, port, q):
    _setup(rank, world, port)
    obj = [bytes(range(128)) if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    q.put((rank, obj[0]))
    dist.destroy_process_group()


def test_unique_id_broadcast():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_id_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(b == bytes(range(128)) for _, b in got)


def test_rccl_unique_id_is_128_bytes():
    from distributed_ddpg_amd.learner import rccl_unique_id
    a, b = rccl_unique_id(), rccl_unique_id()
    assert len(a) == 128 and a != b


@pytest.mark.parametrize("world", [2, 4, 8])
def test_global_draw_sharding(world):
    """Every rank runs the same sampler; slices partition the 1-rank batch."""
    from distributed_ddpg_amd.replay_buffer import Sampler
    Bg = 4096 * world // 4
    full = Sampler(1234).sample(1_000_000, Bg)
    shards = []
    for r in range(world):
        draw = Sampler(1234).sample(1_000_000, Bg)
        b = Bg // world
        shards.append(draw[r * b:(r + 1) * b])
    assert np.array_equal(np.concatenate(shards), full)
    assert len(set(full.tolist())) == Bg
