"""Data parallelism with N real ranks on ONE GPU (replaces the
reference's parameter-server push, ddpg.py:168-174, networks.py:44,137).

RCCL refuses two ranks on one device, so these tests run the library variant
tools/shm/libddpg_shm.so -- the product objects linked against a /dev/shm
stand-in for the RCCL calls (tools/rccl_shm.cpp: host-synchronous, every
reduction in rank order).  Everything else is the product's data-parallel
path: each rank's slice of the global MT19937 draw, its partial gradients,
the exchange call sites and buffers of csrc/dp.hip (fp32 all-reduce; the bf16
configuration's fp32 reduce-scatter, one bf16 rounding, bf16 all-gather, with
the n % N tail all-reduced; the stats all-gather and ordered reduction), the
replicated Adam and soft update, the small-batch path's split gradient / Adam
launches.  Checks:

  * every rank ends every step with the same bits in all ten buffers
    (parameters, targets, Adam slots, gradients);
  * after one step the exchanged gradients, Adam slots and stats equal the
    single-process step on the whole global batch (world 1, product library)
    within the fp32 bar (1e-4) -- the bf16 bars for the bf16 configuration.

RCCL's own transport at N >= 2 is not what runs here (no second GPU).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from test_gpu_parity import GRAD_TOL, rel

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "dp_shm_worker.py")
SHM_LIB = os.path.join(ROOT, "tools", "shm", "libddpg_shm.so")
STEPS = 3


def _env(extra):
    env = dict(os.environ)
    for k in ("DDPG_LIB_PATH", "DDPG_GRAPH_COMM", "RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    env.update(extra)
    return env


def _run(cfg, dtype, b, world, tmp_path, port):
    outs = [str(tmp_path / ("r%d.npz" % r)) for r in range(world)]
    procs = []
    for r in range(world):
        env = _env({"RANK": str(r), "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port), "DDPG_LIB_PATH": SHM_LIB, "DDPG_GRAPH_COMM": "0"})
        procs.append(subprocess.Popen([sys.executable, WORKER, cfg, dtype, str(b), str(STEPS),
                                       outs[r]], env=env, cwd=ROOT))
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=300))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert rcs == [0] * world, rcs
    ref = str(tmp_path / "ref.npz")
    rc = subprocess.run([sys.executable, WORKER, cfg, dtype, str(b * world), "1", ref],
                        env=_env({"RANK": "0", "WORLD_SIZE": "1"}), cwd=ROOT, timeout=300).returncode
    assert rc == 0
    return [np.load(o) for o in outs], np.load(ref)


def _normrel(x, r):
    x = np.asarray(x, np.float64)
    r = np.asarray(r, np.float64)
    return float(np.linalg.norm(x - r) / max(np.linalg.norm(r), 1e-30))


@pytest.mark.parametrize("cfg,dtype,b,world,port", [
    ("c3", "fp32", 256, 2, 29611),   # large-batch path, fp32 all-reduce
    ("c2", "fp32", 64, 2, 29612),    # small-batch path under a communicator
    ("c5", "bf16", 256, 4, 29613),   # bf16 configuration: reduce-scatter + bf16 all-gather
])
def test_dp_ranks_on_one_gpu(cfg, dtype, b, world, port, tmp_path):
    assert os.path.exists(SHM_LIB), "build it: tools/build_shm_variant.sh (build() does)"
    ranks, ref = _run(cfg, dtype, b, world, tmp_path, port)
    assert str(ref["lib"]) == "libddpg_hip.so"
    for r in ranks:
        assert str(r["lib"]) == "libddpg_shm.so"
        # eager steps (the stand-in cannot be graph-captured), none failed over
        assert int(r["counts"][0]) == 0 and int(r["counts"][1]) == STEPS and int(r["counts"][2]) == 0
    # replicated state: identical bits on every rank, first and last step
    for k in ranks[0].files:
        if k == "lib":
            continue
        for r in ranks[1:]:
            assert np.array_equal(ranks[0][k], r[k]), k
    got = ranks[0]
    # each rank's own partial gradient differs from the exchanged sum: the
    # agreement above is the exchange's doing, the check below its value
    # the global-batch step of one process (stats: max Q over ranks, loss summed)
    sq, sl = got["stats0"]
    rq, rl = ref["stats0"]
    assert abs(sq - rq) <= 1e-5 * max(1.0, abs(rq)), (sq, rq)
    assert abs(sl - rl) <= GRAD_TOL * abs(rl), (sl, rl)
    # gradients (8: actor, 9: critic) and Adam slots after step 1
    for w in (8, 9, 4, 6):
        g, r = got["s0_w%d" % w], ref["s0_w%d" % w]
        if dtype == "fp32":
            assert rel(g, r) < GRAD_TOL, (w, rel(g, r))
        else:
            from test_gpu_configs import BF16_GRAD_NORM_TOL
            assert _normrel(g, r) < BF16_GRAD_NORM_TOL, (w, _normrel(g, r))
