"""GPU tests of every environment-selected kernel path, of the RCCL call sites
of the data-parallel step (through a 1-rank communicator), and of the bf16
twins after small-batch steps.  All calls go through the C-ABI.

Switches (read at ddpg_create, so each session below sees its own setting):
  placement only -- results must be BITWISE equal to the default:
    DDPG_XCD=0        no XCD-aware tile order
    DDPG_XCD_RECT=0   row-major XCD runs instead of per-XCD tile rectangles
    DDPG_PAR=1        independent branches forked onto two aux streams
    DDPG_SB_XCD=0     small-batch workgroups dealt over the XCDs (the default
                      packs up to 32 of them on one XCD)
    DDPG_L1BATCH=0    the large-batch step's first layers launched per network
                      instead of as one five-part thin_k launch
    DDPG_ACT32=1      fp32 copies of h1 / cat / cat2 written beside their planes
                      (the default reads the EluGrad operand from the planes)
    DDPG_GEMM_H3=0    twin GEMMs with runtime ring-slot addressing (gemm_h_kernel,
                      gemm_h16_kernel) instead of gemm_h3_kernel / gemm_h16i_kernel
                      (gemm_h3.h): same products, same order (fp32 and bf16;
                      both on the unsplit plan, DDPG_KCOMB=0, since only the
                      gemm_h3.h kernels combine in-launch K splits; fp32 with
                      DDPG_GEMM_M16=0 on both sides, the 32x32x16 forms)
    DDPG_TK_RPB=3     thin_k blocks walk 3 row tiles each (W panel staged once,
                      next X tile prefetched) instead of the automatic count
    DDPG_GEMM_PACK=0  the bf16 configuration's S > 64 first layers launched one
                      by one instead of as one gemm_hw_pack_kernel launch
                      (gemm_h16i_pack_kernel with DDPG_GEMM_HW=0)
    DDPG_TK_FWD=0     thin_k's forward and backward parts on the generic epilogue
                      instead of the forward / backward forms (same arithmetic,
                      flags and bounds folded away)
    DDPG_SKINNY_NL=0  the skinny weight-gradient kernel reads each narrow row by
                      scalar loads instead of from the split's rows staged in LDS
    DDPG_SLOTS_H2D=1  the step's replay slots uploaded to device memory first
                      instead of read in place from the pinned host buffer
  different kernels -- the oracle's fp32 bars (1e-4 after the fused steps):
    DDPG_GEMM=f32     every GEMM on the fp32-input MFMA kernel (no twins)
    DDPG_GEMM_H=0     no twins; large GEMMs on gemm_s3 (operands split while staging)
    DDPG_THINK=0      the K <= 64 layers on the tiled GEMMs instead of thin_k
    DDPG_SKINNY=0     the <= 64-wide weight gradients on the GEMMs instead of
                      the skinny VALU kernel
    DDPG_NW_FUSE=0    dW1 / dWs / dWa on the skinny kernel instead of the dz1 /
                      dcat GEMM epilogues
    DDPG_GEMM_M16=0   the fp32 forward / dX twin GEMMs on gemm_h3_kernel
                      (32x32x16 MFMA) instead of gemm_h3m_kernel (16x16x32:
                      32 products per MFMA instead of 16, fp32 rounding differs)
  bf16 configuration, different summation order -- the oracle's bf16 bars,
  and the two paths' gradients against each other:
    DDPG_GEMM_HW=0    the weight gradients on gemm_h16_kernel instead of
                      gemm_hw_kernel (128 x 64 wave tiles, gemm_hw.h)
    DDPG_GEMM256=1    the split-K weight gradients on the 256 x 256-tile GEMM
                      (gemm_h256.h) instead of gemm_h16_kernel
"""
import random

import numpy as np
import pytest

from test_gpu_parity import (CONFIGS, GRAD_TOL, FWD_TOL, _batch, _fill, _params, _session,
                             _session_dtype, assert_steps_close, f64, rel)

pytestmark = pytest.mark.gpu

SWITCHES = ("DDPG_XCD", "DDPG_XCD_RECT", "DDPG_PAR", "DDPG_SB_XCD", "DDPG_GEMM",
            "DDPG_GEMM_H", "DDPG_THINK", "DDPG_GRAPH", "DDPG_SMALL", "DDPG_SKINNY", "DDPG_L1BATCH",
            "DDPG_ACT32", "DDPG_GEMM256", "DDPG_GEMM_H3", "DDPG_TK_RPB",
            "DDPG_SLOTS_H2D", "DDPG_GRAPH_AUTO", "DDPG_KCOMB", "DDPG_KCOMB_BLOCKS",
            "DDPG_GRAPH_COMM", "DDPG_TEST_CS_SPIN", "DDPG_KCOMB_SPLITS", "DDPG_TK_FWD",
            "DDPG_PROF_SHAPES", "DDPG_GEMM_PACK", "DDPG_HALF_TWIN", "DDPG_SKINNY_NL",
            "DDPG_GEMM_M16", "DDPG_NW_FUSE", "DDPG_KCOMB_WGRAD", "DDPG_GEMM_HW",
            "DDPG_FWD_PACK", "DDPG_GATHER16", "DDPG_PRED_SPIN",
            "DDPG_STATS_SPIN", "DDPG_RING_ARGS")


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


def _clear(monkeypatch):
    for k in SWITCHES:
        monkeypatch.delenv(k, raising=False)


def _run(dd, O, name, p, steps, dtype="fp32", seed=2, profile=False, comm=False):
    """`steps` fused steps on a fresh session; returns the final state, the
    per-step stats and (profile=True) the profiled kernel keys."""
    from distributed_ddpg_amd import _lib
    from distributed_ddpg_amd.learner import FusedLearner, Profile, init_comm
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    S, A, H1, H2, scale, B, _ = CONFIGS[name]
    if dtype == "fp32":
        sess, actor, critic = _session(dd, O, name, p)
    else:
        sess, actor, critic = _session_dtype(dd, O, name, p, dtype)
    if comm:
        init_comm(sess, 0, 1, single=True)
    rb = ReplayBuffer(5000, 1234)
    rows = _fill(rb, S, A, 3000, scale, seed=seed)
    fl = FusedLearner(sess, rb, B)
    prof = Profile(sess)
    if profile:
        prof.enable(True)
    st = [fl.step(stats=True) for _ in range(steps)]
    prof_rows = prof.read() if profile else {}
    keys = sorted(prof_rows)
    if profile:
        prof.enable(False)
    state = [sess.get_params(w) for w in (_lib.ACTOR, _lib.CRITIC, _lib.ACTOR_TARGET,
                                          _lib.CRITIC_TARGET, _lib.ACTOR_ADAM_M, _lib.ACTOR_ADAM_V,
                                          _lib.CRITIC_ADAM_M, _lib.CRITIC_ADAM_V, _lib.ACTOR_GRAD,
                                          _lib.CRITIC_GRAD)]
    powers = (sess.get_adam_powers(0), sess.get_adam_powers(1))
    acc = fl.read_stats()
    sess.close()
    return {"state": state, "stats": st, "powers": powers, "acc": acc, "keys": keys,
            "rows": rows, "prof": prof_rows}


def _bitwise(a, b):
    assert a["stats"] == b["stats"]
    assert a["powers"] == b["powers"]
    assert a["acc"] == b["acc"]
    for x, y in zip(a["state"], b["state"]):
        for u, v in zip(x, y):
            assert np.array_equal(u, v)


def _oracle(O, name, p, rows, steps):
    S, A, H1, H2, scale, B, _ = CONFIGS[name]
    L = O.Learner(S, A, H1, H2, scale, dtype=np.float64, params=p, init_blend=False)
    L32 = O.Learner(S, A, H1, H2, scale, dtype=np.float32, params=p, init_blend=False)
    rr = random.Random(1234)
    for _ in range(steps):
        idx = np.array(rr.sample(range(3000), B))
        L.step(*(x[idx] for x in rows))
        L32.step(*(x[idx] for x in rows))
    return L, L32


@pytest.mark.parametrize("switch,value,name", [
    ("DDPG_XCD", "0", "wide"),
    ("DDPG_XCD_RECT", "0", "wide"),
    ("DDPG_PAR", "1", "wide"),
    ("DDPG_SB_XCD", "0", "ip"),
    ("DDPG_L1BATCH", "0", "wide"),
    ("DDPG_ACT32", "1", "wide"),
    ("DDPG_GEMM_H3", "0", "wide"),
    ("DDPG_TK_RPB", "3", "wide"),
    ("DDPG_TK_FWD", "0", "wide"),
    ("DDPG_SKINNY_NL", "0", "wide"),
    ("DDPG_SLOTS_H2D", "1", "wide"),
    ("DDPG_SLOTS_H2D", "1", "ip"),
    ("DDPG_GATHER16", "0", "wide"),
    ("DDPG_GATHER16", "0", "wides"),
])
def test_placement_switch_bitwise(dd, O, monkeypatch, switch, value, name):
    _clear(monkeypatch)
    if switch == "DDPG_GEMM_H3":
        # gemm_h_kernel has no in-launch K split (small-M plan): compare both
        # kernels on the same unsplit plan; and the 32x32x16 forms on both
        # sides (gemm_h3_kernel vs gemm_h_kernel: same products, same order)
        monkeypatch.setenv("DDPG_KCOMB", "0")
        monkeypatch.setenv("DDPG_GEMM_M16", "0")
        # the fused narrow weight gradients run in gemm_h3's epilogue only
        monkeypatch.setenv("DDPG_NW_FUSE", "0")
    if switch == "DDPG_SKINNY_NL":  # the skinny kernel runs only unfused
        monkeypatch.setenv("DDPG_NW_FUSE", "0")
    p, _ = _params(O, name)
    ref = _run(dd, O, name, p, 3, profile=switch == "DDPG_TK_FWD")
    monkeypatch.setenv(switch, value)
    got = _run(dd, O, name, p, 3, profile=switch == "DDPG_TK_FWD")
    if switch == "DDPG_TK_FWD":  # the default runs both forms, the switch neither
        for form in ("<FWD>", "<BWD>"):
            assert any(k.startswith("thin_k_kernel" + form) for k in ref["keys"]), ref["keys"]
        assert not any(k.startswith(("thin_k_kernel<FWD>", "thin_k_kernel<BWD>"))
                       for k in got["keys"]), got["keys"]
    _bitwise(got, ref)


def test_tk_fwd_bf16_bitwise(dd, O, monkeypatch):
    """bf16 configuration (fp32 activation copies beside the bf16 twins): the
    thin_k forward form with its fp32 copy against the generic epilogue
    (DDPG_TK_FWD=0) -- bitwise after 2 fused steps."""
    _clear(monkeypatch)
    p, _ = _params(O, "wide")
    ref = _run(dd, O, "wide", p, 2, dtype="bf16", profile=True)
    assert any(k.startswith("thin_k_kernel<FWD>") for k in ref["keys"]), ref["keys"]
    monkeypatch.setenv("DDPG_TK_FWD", "0")
    got = _run(dd, O, "wide", p, 2, dtype="bf16", profile=True)
    assert not any(k.startswith("thin_k_kernel<FWD>") for k in got["keys"]), got["keys"]
    _bitwise(got, ref)


def test_gemm_pack_bf16_bitwise(dd, O, monkeypatch):
    """bf16 configuration with S = 200 (first layers on the GEMMs): the four
    batch-only K = S first layers as one gemm_hw_pack_kernel launch by
    default (two 4-wave 128 x 64-wave-tile blocks per CU, gemm_hw.h), as one
    gemm_h16i_pack_kernel launch with DDPG_GEMM_HW=0, and one
    gemm_h16i_kernel launch each with DDPG_GEMM_PACK=0 -- the same 16x16x32
    MFMAs per output over the same k order and the same epilogue ops: bitwise
    equal after 2 fused steps.  DDPG_KCOMB=0 keeps B = 256 on the unsplit plan
    the pack takes."""
    _clear(monkeypatch)
    monkeypatch.setenv("DDPG_KCOMB", "0")
    p, _ = _params(O, "wides")
    ref = _run(dd, O, "wides", p, 2, dtype="bf16", profile=True)
    assert any(k.startswith("gemm_hw_pack_kernel") for k in ref["keys"]), ref["keys"]
    monkeypatch.setenv("DDPG_GEMM_HW", "0")
    got_h16 = _run(dd, O, "wides", p, 2, dtype="bf16", profile=True)
    assert any(k.startswith("gemm_h16i_pack_kernel") for k in got_h16["keys"]), got_h16["keys"]
    monkeypatch.setenv("DDPG_GEMM_HW", "1")
    monkeypatch.setenv("DDPG_GEMM_PACK", "0")
    got = _run(dd, O, "wides", p, 2, dtype="bf16", profile=True)
    assert not any("pack_kernel" in k for k in got["keys"]), got["keys"]
    _bitwise(got_h16, ref)
    _bitwise(got, ref)


@pytest.mark.parametrize("name,dtype,kern", [("wide", "fp32", "gemm_h3m_pack_kernel"),
                                              ("wides", "bf16", "gemm_h16i_pack_kernel")])
def test_fwd_pack_bitwise(dd, O, monkeypatch, name, dtype, kern):
    """The step's three forward layers that read only the first layers'
    outputs (target actor W2, online actor W2, online critic Wh) as one pack
    launch by default, and in the sequential order with DDPG_FWD_PACK=0: the
    same kernel body per tile, the same buffers -- bitwise equal after 2 fused
    steps.  DDPG_KCOMB=0 keeps B = 256 on the unsplit plan the pack takes."""
    _clear(monkeypatch)
    monkeypatch.setenv("DDPG_KCOMB", "0")
    p, _ = _params(O, name)
    ref = _run(dd, O, name, p, 2, dtype=dtype, profile=True)
    assert any(k.startswith(kern) and k.endswith("|fwd_head") for k in ref["keys"]), ref["keys"]
    monkeypatch.setenv("DDPG_FWD_PACK", "0")
    got = _run(dd, O, name, p, 2, dtype=dtype, profile=True)
    assert not any(k.endswith("|fwd_head") and "pack_kernel" in k for k in got["keys"]), got["keys"]
    _bitwise(got, ref)


def test_half_twin_bf16_bitwise(dd, O, monkeypatch):
    """bf16 configuration, S = 200: the state halves of cat2 (critic at
    (s, mu)) and of dcat (read by dWs through its twin) are stored as bf16
    twins only by default -- their fp32 values have no reader -- and in fp32
    too with DDPG_HALF_TWIN=0: bitwise equal."""
    _clear(monkeypatch)
    p, _ = _params(O, "wides")
    ref = _run(dd, O, "wides", p, 2, dtype="bf16")
    monkeypatch.setenv("DDPG_HALF_TWIN", "0")
    got = _run(dd, O, "wides", p, 2, dtype="bf16")
    _bitwise(got, ref)


def test_gemm_h3_switch_bf16_bitwise(dd, O, monkeypatch):
    """bf16 configuration: the forward / dX GEMMs on gemm_h16i_kernel (per-tile
    slot base + immediate offsets, gemm_h3.h) by default and on
    gemm_h16_kernel with DDPG_GEMM_H3=0 -- same products in the same order,
    bitwise equal results after 2 fused steps (the narrow weight gradients on
    the skinny kernel on both sides: gemm_h16_kernel has no fused form)."""
    _clear(monkeypatch)
    monkeypatch.setenv("DDPG_KCOMB", "0")  # gemm_h16_kernel has no in-launch K split
    monkeypatch.setenv("DDPG_NW_FUSE", "0")
    monkeypatch.setenv("DDPG_GEMM_HW", "0")  # the weight gradients on gemm_h16_kernel both sides
    p, _ = _params(O, "wide")
    ref = _run(dd, O, "wide", p, 2, dtype="bf16", profile=True)
    assert any(k.startswith("gemm_h16i_kernel<RK,KR") for k in ref["keys"]), ref["keys"]
    assert any(k.startswith("gemm_h16i_kernel<RK,RK") for k in ref["keys"]), ref["keys"]
    monkeypatch.setenv("DDPG_GEMM_H3", "0")
    got = _run(dd, O, "wide", p, 2, dtype="bf16", profile=True)
    assert not any(k.startswith("gemm_h16i_kernel") for k in got["keys"]), got["keys"]
    _bitwise(got, ref)


def test_gemm256_switch_bf16(dd, O, monkeypatch):
    """bf16 configuration at the 1024-wide config (B = 256): with
    DDPG_GEMM256=1 the split-K weight gradients dWh (2048 x 1024) and dW2
    (1024 x 1024) run on gemm_h256_kernel (MODE 0, whole 256 x 256 tiles); by
    default (measured slower in the step) on gemm_h16_kernel.  The
    products are the same bf16 values with fp32 accumulation in another
    order: the first step's critic gradients agree to 1e-5 norm-wise (the
    actor's, taken through the UPDATED critic whose Adam step can flip on
    near-zero gradients, to 1e-3), and both runs' parameters after 3 fused
    steps meet the oracle's stated bf16 bar (BF16_PARAM_TOL)."""
    from test_gpu_parity import BF16_PARAM_TOL, normrel
    _clear(monkeypatch)
    monkeypatch.setenv("DDPG_GEMM_HW", "0")  # gemm_h16_kernel is the reference side
    name = "wide"
    p, _ = _params(O, name)
    ref1 = _run(dd, O, name, p, 1, dtype="bf16")
    ref = _run(dd, O, name, p, 3, dtype="bf16", profile=True)
    assert not any(k.startswith("gemm_h256_kernel") for k in ref["keys"]), ref["keys"]
    assert any(k.startswith("gemm_h16_kernel<KR,KR") for k in ref["keys"]), ref["keys"]
    monkeypatch.setenv("DDPG_GEMM256", "1")
    got1 = _run(dd, O, name, p, 1, dtype="bf16")
    got = _run(dd, O, name, p, 3, dtype="bf16", profile=True)
    assert "gemm_h256_kernel<KR,KR,MODE=0>|wgrad" in got["keys"], got["keys"]
    for bar, x, y in zip((1e-3, 1e-5), ref1["state"][8:], got1["state"][8:]):  # actor, critic
        for u, v in zip(x, y):
            assert normrel(v, u) < bar, normrel(v, u)
    L, _ = _oracle(O, name, p, ref["rows"], 3)
    for run in (ref, got):
        for (net, keys), vals in zip((("actor", O.ACTOR_KEYS), ("critic", O.CRITIC_KEYS)),
                                     run["state"][:2]):
            for k, v in zip(keys, vals):
                assert rel(v, L.state()[net][k].reshape(v.shape)) < BF16_PARAM_TOL, (net, k)


def test_gemm_hw_weight_gradients_bf16(dd, O, monkeypatch):
    """bf16 configuration at the 1024-wide config (B = 256): the weight
    gradients dWh (2048 x 1024) and dW2 (1024 x 1024) run on gemm_hw_kernel
    (256 x 128 tiles, 128 x 64 wave tiles, gemm_hw.h) by default and on
    gemm_h16_kernel with DDPG_GEMM_HW=0.  The same bf16 products with fp32
    accumulation in another order: the first step's critic gradients agree
    to 1e-5 norm-wise (the actor's, through the UPDATED critic, to 1e-3), and
    both runs' parameters after 3 fused steps meet the oracle's bf16 bar."""
    from test_gpu_parity import BF16_PARAM_TOL, normrel
    name = "wide"
    runs = {}
    for hw in ("1", "0"):
        _clear(monkeypatch)
        monkeypatch.setenv("DDPG_GEMM_HW", hw)
        p, _ = _params(O, name)
        runs[hw] = (_run(dd, O, name, p, 1, dtype="bf16"),
                    _run(dd, O, name, p, 3, dtype="bf16", profile=True))
    keys = {hw: [k for k in r[1]["keys"] if "<KR,KR" in k] for hw, r in runs.items()}
    assert keys["1"] and all(k.startswith("gemm_hw_kernel<KR,KR,NP=1>") for k in keys["1"]), keys
    assert keys["0"] and all(k.startswith("gemm_h16_kernel<KR,KR") for k in keys["0"]), keys
    for bar, x, y in zip((1e-3, 1e-5), runs["0"][0]["state"][8:], runs["1"][0]["state"][8:]):
        for u, v in zip(x, y):
            assert normrel(v, u) < bar, normrel(v, u)
    L, _ = _oracle(O, name, p, runs["1"][1]["rows"], 3)
    for _, run in runs.values():
        for (net, keys_), vals in zip((("actor", O.ACTOR_KEYS), ("critic", O.CRITIC_KEYS)),
                                      run["state"][:2]):
            for k, v in zip(keys_, vals):
                assert rel(v, L.state()[net][k].reshape(v.shape)) < BF16_PARAM_TOL, (net, k)


@pytest.mark.parametrize("switch,value,kernel,absent", [
    ("DDPG_GEMM", "f32", "gemm_f32_kernel", "gemm_h"),
    ("DDPG_GEMM_H", "0", "gemm_s3_kernel", "gemm_h"),
    ("DDPG_THINK", "0", "gemm_h3m_kernel", "thin_k_kernel"),
    ("DDPG_GEMM_M16", "0", "gemm_h3_kernel<RK,KR", "gemm_h3m_kernel"),
    ("DDPG_SKINNY", "0", "gemm_f32_kernel", "skinny_wgrad_kernel"),
])
def test_kernel_switch_oracle(dd, O, monkeypatch, switch, value, kernel, absent):
    """A switch that selects different kernels: 3 fused steps at the 1024-wide
    config still meet the oracle's fp32 bars, on the kernels it names."""
    _clear(monkeypatch)
    monkeypatch.setenv(switch, value)
    if switch == "DDPG_SKINNY":  # every narrow weight gradient is fused by default
        monkeypatch.setenv("DDPG_NW_FUSE", "0")
    name = "wide"
    p, _ = _params(O, name)
    got = _run(dd, O, name, p, 3, profile=True)
    assert any(k.startswith(kernel) for k in got["keys"]), got["keys"]
    assert not any(k.startswith(absent) for k in got["keys"]), got["keys"]
    L, L32 = _oracle(O, name, p, got["rows"], 3)
    nets = (("actor", O.ACTOR_KEYS), ("critic", O.CRITIC_KEYS), ("actor_t", O.ACTOR_KEYS),
            ("critic_t", O.CRITIC_KEYS))
    for (net, keys), vals in zip(nets, got["state"][:4]):
        for k, v in zip(keys, vals):
            assert_steps_close(v, L.state()[net][k], L32.state()[net][k], (switch, net, k))


@pytest.mark.parametrize("fuse", ["1", "0"])
def test_narrow_wgrad_fused_into_dx(dd, O, monkeypatch, fuse):
    """dW1 = s^T dz1, dWs = s^T dcat_s, dWa = a^T dcat_a (narrow side <= 64)
    computed in the dz1 / dcat GEMM epilogues (per-row-tile fp32 partials
    summed with the other slabs) and dW3 = h2^T dz3 in the dz2 thin_k launch
    by default, and on the skinny kernel with DDPG_NW_FUSE=0 (four launches):
    both meet the oracle's fp32 bars after 3 fused steps at the 1024-wide
    config."""
    _clear(monkeypatch)
    if fuse == "0":
        monkeypatch.setenv("DDPG_NW_FUSE", "0")
    p, _ = _params(O, "wide")
    got = _run(dd, O, "wide", p, 3)
    L, L32 = _oracle(O, "wide", p, got["rows"], 3)
    nets = (("actor", O.ACTOR_KEYS), ("critic", O.CRITIC_KEYS))
    for (net, keys), vals in zip(nets, got["state"][:2]):
        for k, v in zip(keys, vals):
            assert_steps_close(v, L.state()[net][k], L32.state()[net][k], (fuse, net, k))


def test_narrow_wgrad_fused_bf16(dd, O, monkeypatch):
    """bf16 configuration with S = 200 > 64, A = 16: dWa = a^T dcat_a in the
    dcat GEMM's epilogue (gemm_h16i_kernel, two 128-row passes per 256-row
    tile, one fp32 partial per 128 rows) and dcat then stored as its bf16 twin
    only (dWs reads the twin); DDPG_NW_FUSE=0: dWa on the skinny kernel from
    the fp32 dcat.  The same fp32 values summed in another order: the first
    step's critic gradients agree to 1e-5 norm-wise, no skinny launch (dW3 in
    the dz2 thin_k launch) instead of two per step, and both runs meet the
    oracle's bf16 bar after 3 fused steps."""
    from test_gpu_parity import BF16_PARAM_TOL, normrel
    name = "wides"
    runs = {}
    for fuse in ("1", "0"):
        _clear(monkeypatch)
        monkeypatch.setenv("DDPG_NW_FUSE", fuse)
        p, _ = _params(O, name)
        first = _run(dd, O, name, p, 1, dtype="bf16")
        run = _run(dd, O, name, p, 3, dtype="bf16", profile=True)
        runs[fuse] = (first, run)
    L, _ = _oracle(O, name, p, runs["1"][1]["rows"], 3)
    for u, v in zip(runs["0"][0]["state"][9], runs["1"][0]["state"][9]):  # critic gradients
        assert normrel(v, u) < 1e-5, normrel(v, u)
    for fuse, (_, run) in runs.items():
        for (net, keys), vals in zip((("actor", O.ACTOR_KEYS), ("critic", O.CRITIC_KEYS)),
                                     run["state"][:2]):
            for k, v in zip(keys, vals):
                assert rel(v, L.state()[net][k].reshape(v.shape)) < BF16_PARAM_TOL, (fuse, net, k)
    skinny = {f: sum(v["launches"] for k, v in r["prof"].items()
                     if k.startswith("skinny_wgrad_kernel")) for f, (_, r) in runs.items()}
    assert skinny == {"1": 0, "0": 6}, skinny


def test_narrow_wgrad_launch_counts(dd, O, monkeypatch):
    """The fused forms really ran: per fused step no skinny launch by default
    (dW1 / dWs / dWa in the dX GEMM epilogues, dW3 in the dz2 thin_k launch),
    4 with DDPG_NW_FUSE=0."""
    from distributed_ddpg_amd.learner import FusedLearner, Profile
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    counts = {}
    for fuse in ("1", "0"):
        _clear(monkeypatch)
        monkeypatch.setenv("DDPG_NW_FUSE", fuse)
        p, _ = _params(O, "wide")
        S, A, H1, H2, scale, B, _ = CONFIGS["wide"]
        sess, actor, critic = _session(dd, O, "wide", p)
        rb = ReplayBuffer(5000, 1234)
        _fill(rb, S, A, 3000, scale, seed=2)
        fl = FusedLearner(sess, rb, B)
        prof = Profile(sess)
        prof.enable(True)
        fl.step()
        keys = prof.read()
        prof.enable(False)
        sess.close()
        counts[fuse] = keys.get("skinny_wgrad_kernel|wgrad", {"launches": 0})["launches"]
    assert counts == {"1": 0, "0": 4}, counts


def test_default_path_uses_skinny_wgrad(dd, O, monkeypatch):
    """The <= 64-wide weight gradients (dW1, dWs, dWa, dW3 at S = 64, A = 16)
    run on skinny_wgrad_kernel when not fused into their producers
    (DDPG_NW_FUSE=0), and the 3-step oracle bars hold."""
    _clear(monkeypatch)
    monkeypatch.setenv("DDPG_NW_FUSE", "0")
    p, _ = _params(O, "wide")
    got = _run(dd, O, "wide", p, 3, profile=True)
    assert "skinny_wgrad_kernel|wgrad" in got["keys"], got["keys"]
    L, L32 = _oracle(O, "wide", p, got["rows"], 3)
    for (net, keys), vals in zip((("actor", O.ACTOR_KEYS), ("critic", O.CRITIC_KEYS)),
                                 got["state"][:2]):
        for k, v in zip(keys, vals):
            assert_steps_close(v, L.state()[net][k], L32.state()[net][k], (net, k))


def test_single_rank_communicator_matches_no_communicator(dd, O, monkeypatch):
    """The data-parallel exchange through RCCL (ncclAllReduce of the critic's
    dWh then the rest, the stats ncclAllGather + stats_reduce_kernel, the
    actor's dW2 then the rest, all on the comm stream) with a 1-rank
    communicator is an identity: gradients, Adam slots, parameters, stats and
    the running sums equal the communicator-less step BITWISE.  B = 1024 keeps
    both runs on the large-batch path (a communicator always takes it).  The
    communicator run combines its weight gradients' K splits in-launch, the
    other sums the same splits as slabs inside its Adam passes."""
    _clear(monkeypatch)
    name = "wide"
    p, _ = _params(O, name)
    S, A, H1, H2, scale, _, src = CONFIGS[name]
    CONFIGS["wide_b1024"] = (S, A, H1, H2, scale, 1024, src)
    try:
        ref = _run(dd, O, "wide_b1024", p, 3, profile=True)
        got = _run(dd, O, "wide_b1024", p, 3, profile=True, comm=True)
    finally:
        del CONFIGS["wide_b1024"]
    assert not any(k.startswith("rccl") for k in ref["keys"]), ref["keys"]
    assert "rccl_allreduce" in got["keys"] and "rccl_stats" in got["keys"], got["keys"]
    assert any(k.endswith("wgrad/kc") for k in got["keys"]), got["keys"]
    assert not any(k.endswith("wgrad/kc") for k in ref["keys"]), ref["keys"]
    assert "adam+reduce+soft_update" in ref["keys"], ref["keys"]
    _bitwise(got, ref)


def test_twins_current_after_small_path_graph_steps(dd, O, monkeypatch):
    """Small-batch fused steps (hipGraph-replayed, B = 64) move theta / theta'
    without their bf16 twins; the next large-batch call must rebuild them.
    Several replays, then predict / predict_target / critic.predict at
    B = 256 (the twin GEMM path) against the oracle on the current params."""
    from distributed_ddpg_amd import _lib
    from distributed_ddpg_amd.learner import FusedLearner
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    _clear(monkeypatch)
    name = "ip"
    S, A, H1, H2, scale, B, _ = CONFIGS[name]
    p, _ = _params(O, name)
    sess, actor, critic = _session(dd, O, name, p, batch_max=512)
    rb = ReplayBuffer(4000, 3)
    _fill(rb, S, A, 3000, scale, seed=6)
    fl = FusedLearner(sess, rb, B)
    rng = np.random.default_rng(17)
    s = rng.standard_normal((256, S)).astype(np.float32)
    a = (rng.uniform(-1, 1, (256, A)) * scale).astype(np.float32)
    for rounds in range(3):
        # raise the learning signal so the params move well past fp32 rounding
        for _ in range(4):
            fl.step()
        cur = {"actor": dict(zip(O.ACTOR_KEYS, sess.get_params(_lib.ACTOR))),
               "actor_t": dict(zip(O.ACTOR_KEYS, sess.get_params(_lib.ACTOR_TARGET))),
               "critic": dict(zip(O.CRITIC_KEYS, sess.get_params(_lib.CRITIC)))}
        mu = actor.predict(s)
        assert rel(mu, O.actor_forward(f64(cur["actor"]), s.astype(np.float64), scale)[3]) < FWD_TOL
        mut = actor.predict_target(s)
        assert rel(mut, O.actor_forward(f64(cur["actor_t"]), s.astype(np.float64),
                                        scale)[3]) < FWD_TOL
        q = critic.predict(s, a)
        assert rel(q, O.critic_forward(f64(cur["critic"]), s.astype(np.float64),
                                       a.astype(np.float64))[3]) < FWD_TOL
    sess.close()


def test_gradient_sets_are_get_only(dd, O):
    from distributed_ddpg_amd import _lib
    p, _ = _params(O, "ip")
    sess, actor, critic = _session(dd, O, "ip", p)
    for which in (_lib.ACTOR_GRAD, _lib.CRITIC_GRAD):
        g = sess.get_params(which)
        with pytest.raises(RuntimeError, match="get-only"):
            sess.set_params(which, g)
    sess.close()


@pytest.mark.parametrize("name", ["ip", "wide"])
def test_slots_in_place_ring_reuse_pipelined(dd, O, monkeypatch, name):
    """The step's replay slots are read in place from pinned (coherent) host
    memory: a ring of kSlotRing = 4 buffers, each rewritten by the host four
    steps later once its event has fired.  Ten eager steps (DDPG_GRAPH=0)
    issued back to back without a host sync -- a pipelined caller, so the ring
    wraps while earlier steps may still run -- equal the uploaded-slots path
    (DDPG_SLOTS_H2D=1) bitwise.  ip: the small-batch path; wide: large batch."""
    from distributed_ddpg_amd.learner import FusedLearner
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    _clear(monkeypatch)
    monkeypatch.setenv("DDPG_GRAPH", "0")
    p, _ = _params(O, name)
    S, A, H1, H2, scale, B, _ = CONFIGS[name]

    def run():
        sess, actor, critic = _session(dd, O, name, p)
        rb = ReplayBuffer(5000, 1234)
        _fill(rb, S, A, 3000, scale, seed=4)
        fl = FusedLearner(sess, rb, B)
        for _ in range(10):
            fl.step()
        sess.sync()
        out = ([sess.get_params(w) for w in (0, 2, 8, 9)], fl.read_stats())
        sess.close()
        return out

    got = run()
    monkeypatch.setenv("DDPG_SLOTS_H2D", "1")
    ref = run()
    assert got[1] == ref[1]
    for x, y in zip(got[0], ref[0]):
        for u, v in zip(x, y):
            assert np.array_equal(u, v)


@pytest.mark.parametrize("name", ["ip", "odd"])
def test_pred_spin_bitwise(dd, O, monkeypatch, name):
    """Action selection (sb_actor_predict) returns once the host sees every
    block's completion word by default, after hipStreamSynchronize with
    DDPG_PRED_SPIN=0: the same actions, bit for bit -- also when the call
    queues behind an asynchronous fused step (the worker's pipelined loop)."""
    from distributed_ddpg_amd.learner import FusedLearner
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    S, A, H1, H2, scale, B, _ = CONFIGS[name]
    p, _ = _params(O, name)
    st = np.random.default_rng(4).standard_normal((B, S)).astype(np.float32)
    outs = []
    for spin in ("1", "0"):
        _clear(monkeypatch)
        monkeypatch.setenv("DDPG_PRED_SPIN", spin)
        sess, actor, critic = _session(dd, O, name, p)
        rb = ReplayBuffer(5000, 1234)
        _fill(rb, S, A, 3000, scale, seed=2)
        fl = FusedLearner(sess, rb, B)
        got = [actor.predict(st[:1]), actor.predict(st), actor.predict_target(st[:3])]
        for _ in range(3):
            fl.step()  # no stats: nothing waits for it
            got.append(actor.predict(st[:1]))
        got.append(actor.predict(st))
        outs.append(got)
        sess.close()
    for x, y in zip(*outs):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("name", ["ip", "wide"])
def test_stats_spin_bitwise(dd, O, monkeypatch, name):
    """Synchronous stats (fused step with stats, critic.train's loss): by
    default a one-thread kernel writes them to pinned host memory and the host
    polls its completion word, with DDPG_STATS_SPIN=0 a device-to-host copy
    and a stream wait -- the same values and states, bit for bit, including
    stats read right after asynchronous steps."""
    S, A, H1, H2, scale, B, _ = CONFIGS[name]
    p, _ = _params(O, name)
    outs = []
    for spin in ("1", "0"):
        _clear(monkeypatch)
        monkeypatch.setenv("DDPG_STATS_SPIN", spin)
        r = _run(dd, O, name, p, 3)
        from distributed_ddpg_amd.learner import FusedLearner
        from distributed_ddpg_amd.replay_buffer import ReplayBuffer
        sess, actor, critic = _session(dd, O, name, p)
        rb = ReplayBuffer(5000, 1234)
        _fill(rb, S, A, 3000, scale, seed=2)
        fl = FusedLearner(sess, rb, B)
        fl.step()
        fl.step()  # asynchronous, then a synchronous read behind them
        st = fl.step(stats=True)
        s_, a_, _r = _batch(name, seed=6)
        y = np.random.default_rng(6).standard_normal((B, 1)).astype(np.float32)
        q, _, loss = critic.train(s_, a_, y)
        sess.close()
        outs.append((r, st, q, loss))
    (r0, st0, q0, l0), (r1, st1, q1, l1) = outs
    _bitwise(r0, r1)
    assert st0 == st1 and np.array_equal(q0, q1) and l0 == l1


@pytest.mark.parametrize("f64", [False, True])
def test_ring_args_bitwise(dd, O, monkeypatch, f64):
    """A worker's single-row adds (ddpg.py:79-84) interleaved with fused steps,
    the ring wrapping: by default each flush is one kernel whose arguments
    carry the rows (no host wait), with DDPG_RING_ARGS=0 copies from the
    staging plus a stream wait -- the same ring, the same steps, bit for bit;
    and sample_batch returns exactly the rows added (fp32 and float64 rings)."""
    from distributed_ddpg_amd.learner import FusedLearner
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    name = "ip"
    S, A, H1, H2, scale, B, _ = CONFIGS[name]
    p, _ = _params(O, name)
    rng = np.random.default_rng(9)
    n = 700
    dt = np.float64 if f64 else np.float32
    rows = (rng.standard_normal((n, S)).astype(dt), rng.uniform(-3, 3, (n, A)).astype(np.float32),
            rng.standard_normal(n).astype(dt), rng.random(n) < 0.05,
            rng.standard_normal((n, S)).astype(dt))
    outs = []
    for v in ("1", "0"):
        _clear(monkeypatch)
        monkeypatch.setenv("DDPG_RING_ARGS", v)
        sess, actor, critic = _session(dd, O, name, p)
        rb = ReplayBuffer(500, 1234)  # 700 adds: the ring wraps
        fl = FusedLearner(sess, rb, B)
        st = []
        for i in range(n):
            # the reward as a scalar, or as a one-element array (some envs)
            r_i = rows[2][i] if i % 2 else np.array([rows[2][i]])
            rb.add(rows[0][i], rows[1][i], r_i, rows[3][i], rows[4][i])
            if i >= B and i % 3 == 0:
                st.append(fl.step(stats=i % 2 == 0))
        with pytest.raises(ValueError):
            rb.add(rows[0][0][:-1], rows[1][0], 0.0, False, rows[4][0])  # short state
        with pytest.raises(ValueError):
            rb.add(rows[0][0], rows[1][0], np.zeros(2), False, rows[4][0])  # two rewards
        assert rb.size() == 500
        s_b, a_b, r_b, t_b, s2_b, pos = rb.sample_batch(64, return_indices=True)
        ins = (n - rb.size()) + np.asarray(pos)  # insertion index of each sampled row
        assert np.array_equal(s_b, rows[0][ins]) and np.array_equal(s2_b, rows[4][ins])
        assert np.array_equal(a_b, rows[1][ins]) and np.array_equal(t_b, rows[3][ins])
        assert np.array_equal(r_b, rows[2][ins])
        state = [sess.get_params(w) for w in (0, 1, 2, 3)]
        sess.close()
        outs.append((st, state))
    assert outs[0][0] == outs[1][0]
    for x, y in zip(outs[0][1], outs[1][1]):
        for u, w in zip(x, y):
            assert np.array_equal(u, w)


def test_ring_args_two_learners(dd, O, monkeypatch):
    """One replay ring read by two learner contexts (two streams) while a
    worker adds single rows: a flush issued on one learner's stream is joined
    by the other learner's gather and by sample_batch on the ring's own
    stream -- the same results as the copy form (DDPG_RING_ARGS=0), bit for
    bit."""
    from distributed_ddpg_amd.learner import FusedLearner
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    name = "ip"
    S, A, H1, H2, scale, B, _ = CONFIGS[name]
    p, _ = _params(O, name)
    rng = np.random.default_rng(12)
    n = 400
    rows = (rng.standard_normal((n, S)).astype(np.float32),
            rng.uniform(-3, 3, (n, A)).astype(np.float32),
            rng.standard_normal(n).astype(np.float32), rng.random(n) < 0.05,
            rng.standard_normal((n, S)).astype(np.float32))
    outs = []
    for v in ("1", "0"):
        _clear(monkeypatch)
        monkeypatch.setenv("DDPG_RING_ARGS", v)
        s1, _, _ = _session(dd, O, name, p)
        s2, _, _ = _session(dd, O, name, p)
        rb = ReplayBuffer(300, 77)
        f1, f2 = FusedLearner(s1, rb, B), FusedLearner(s2, rb, B)
        st = []
        for i in range(n):
            rb.add(rows[0][i], rows[1][i], rows[2][i], rows[3][i], rows[4][i])
            if i >= B and i % 2 == 0:
                st.append((f1 if i % 4 == 0 else f2).step(stats=True))
        sb = rb.sample_batch(32, return_indices=True)
        state = [x.get_params(w) for x in (s1, s2) for w in (0, 1)]
        s1.close()
        s2.close()
        outs.append((st, sb, state))
    assert outs[0][0] == outs[1][0]
    for x, y in zip(outs[0][1], outs[1][1]):
        assert np.array_equal(x, y)
    for x, y in zip(outs[0][2], outs[1][2]):
        for u, w in zip(x, y):
            assert np.array_equal(u, w)
