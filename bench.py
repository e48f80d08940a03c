"""Benchmark: DDPG actor+critic learner updates/s on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c5|c1]
                  [--scaling weak|strong]

One "step" = one whole learner update (ddpg.py:86-113) as ddpg_learner_step:
host MT19937 draw of the batch from a replay ring filled to 1e6 synthetic
transitions, device gather, target/critic/actor forward and
backward, both Adam updates, both soft updates.  Inputs are resident in HBM
before the timed region.  N>1: one process per GPU (launched by torchrun, or
by this script itself when --gpus N > 1 and WORLD_SIZE is unset: it then
starts N rank processes before touching the GPU and exits with the worst rank
status), synchronous data parallelism, RCCL all-reduce of the critic then actor
gradients.  --scaling weak (default): per-GPU batch fixed at the config's B,
value = batch-B updates processed by all ranks / max-over-ranks time.
--scaling strong: global batch fixed at B (B/N rows per GPU), value = global
updates / s.

Rank 0 prints ONE JSON line with the contract fields plus
  roofline      dominant kernel (HIP-event timed in-process) vs its MFMA peak (fp32:
                157.3 TF; fp32-on-bf16 gemm_s3: 2.5 PF / 6 products), + frac vs fp32 peak
  cpu_baseline  the reference's deque sample_batch + a torch-CPU restatement of its 8
                sess.run calls per step (oracle/torch_cpu.py) on the host cores: 16
                threads and 1 thread; + C2 and C1 (B=64), C2 also at os.cpu_count()
  step_latency  p10 / median / p90 of per-step wall time (host sync after each step)
  small_batch   the InvertedPendulum B=64 latency-bound configuration (N=1 only), with
                action selection (predict on one state) and the worker's per-env-step
                device work (predict + one replay add + a step with stats) in us
  c5_bf16       BASELINE configs[4] (S=376, A=17, 2048-wide, B=4096, bf16) (c3 only; every N)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: Peak FP32 (matrix) 157.3 TF spec
PEAK_HBM_GBS = 8000.0           # 8 TB/s spec

CONFIGS = {
    # name: (S, A, H1, H2, B per GPU, action_scale, label)
    "c3": (64, 16, 1024, 1024, 4096, 1.0,
           "C3 synthetic S=64 A=16 actor/critic 1024/1024, batch 4096/GPU"),
    "c2": (4, 1, 128, 200, 64, 3.0,
           "C2 InvertedPendulum-shaped S=4 A=1 128/200, batch 64"),
    # the reference's own default batch (parameters.py:11)
    "c2b": (4, 1, 128, 200, 256, 3.0,
            "C2 InvertedPendulum-shaped S=4 A=1 128/200, batch 256 (parameters.py:11)"),
    "c5": (376, 17, 2048, 2048, 4096, 1.0,
           "C5 Humanoid-shaped S=376 A=17 2048/2048, batch 4096/GPU"),
    # BASELINE configs[0]: MountainCar-shaped, 400/300 MLP, batch 64 (CPU leg)
    "c1": (2, 1, 400, 300, 64, 1.0,
           "C1 MountainCar-shaped S=2 A=1 400/300, batch 64"),
}
DEFAULT_DTYPE = {"c3": "fp32", "c2": "fp32", "c2b": "fp32", "c5": "bf16", "c1": "fp32"}
PEAK_BF16_MFMA_TFLOPS = 2500.0  # ~2.5 PF dense (MI355X_MICROARCH.md)
# fp32 GEMMs on the bf16 pipe (gemm_s3): six bf16 MFMA products per fp32 MAC,
# so the pipe bounds fp32-equivalent throughput at 2.5 PF / 6
PEAK_S3_FP32EQ_TFLOPS = PEAK_BF16_MFMA_TFLOPS / 6.0
REPLAY_ROWS = 1_000_000


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def spawn_ranks(n):
    """--gpus N > 1 without a launcher: start N rank processes of this script
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, the same
    arguments), before this process touches the GPU.  Rank 0 prints the JSON
    line.  If a rank fails the others are stopped.  Returns the worst exit
    status (0 when every rank succeeded)."""
    import signal
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rcs = [None] * n
    first_bad = None
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        if any(rc not in (None, 0) for rc in rcs):
            bad = [(i, rc) for i, rc in enumerate(rcs) if rc not in (None, 0)]
            first_bad = bad[0][1]
            log("[bench] rank(s) %s failed; stopping the others" % bad)
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.send_signal(signal.SIGTERM)
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    try:
                        rcs[i] = p.wait(timeout=20)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[i] = p.wait()
            break
        time.sleep(0.2)
    # the status of the first rank that failed by itself; signal k -> 128 + k
    rc = first_bad if first_bad is not None else next((r for r in rcs if r), 0)
    return rc if rc >= 0 else 128 - rc


class stdout_to_stderr:
    """Point fd 1 at stderr for the duration (native libraries' banners), so
    that stdout carries only the one JSON line of the bench contract."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def build_learner(cfg_name, device, rank, world, replay_rows, seed=1234, dtype="fp32",
                  per_gpu_b=None, rb=None, proxy=False):
    """Session + replay ring (filled, or `rb` reused) + fused learner.
    proxy: world > 1 on ONE GPU -- rank `rank`'s share of a world-rank step
    with a 1-rank stand-in communicator (ddpg_comm_init_proxy)."""
    from distributed_ddpg_amd import _lib, networks as nets
    from distributed_ddpg_amd.learner import FusedLearner, fill_synthetic, init_comm
    from distributed_ddpg_amd.replay_buffer import ReplayBuffer
    S, A, H1, H2, B, scale, _ = CONFIGS[cfg_name]
    B = per_gpu_b or B
    nets.reset_default_graph()
    actor = nets.ActorNetwork(S, A, scale, 1e-4, 1e-3, None, h1=H1, h2=H2)
    critic = nets.CriticNetwork(S, A, 1e-3, 1e-3, actor.get_num_trainable_vars(), None, h1=H1,
                                h2=H2)
    sess = nets.Session(device=device, batch_max=B, rank=rank, world=world, dtype=dtype)
    actor.set_session(sess)
    critic.set_session(sess)
    sess.run(nets.global_variables_initializer(seed=seed))   # same init on every rank
    actor.update_target_network()                            # ddpg.py:228-229
    critic.update_target_network()
    with stdout_to_stderr():   # RCCL prints a version banner on fd 1 at init
        if proxy:
            _lib.check(_lib.lib.ddpg_comm_init_proxy(sess.ctx), sess.ctx)
        else:
            init_comm(sess, rank, world)
    if rb is None:
        rb = ReplayBuffer(replay_rows, seed, device=device)
        t0 = time.time()
        fill_synthetic(rb, S, A, replay_rows, scale=scale, seed=seed)   # identical on every rank
        log("[bench] rank %d replay filled with %d rows in %.1fs" % (rank, replay_rows,
                                                                     time.time() - t0))
    return sess, rb, FusedLearner(sess, rb, B * world), actor


# ---------------------------------------------------------------- projected scaling
# Exchange model for the N-GPU projection.  Stated inputs, not
# measurements: xGMI links of ~153 GB/s bidirectional, taken as 64 GB/s
# effective per direction; a ring all-reduce over N GPUs of one node uses the
# N-1 direct links of each GPU, at RCCL_EFF of their sum (bus bandwidth); a
# fixed latency per collective call.
XGMI_LINK_GBS = 64.0
RCCL_EFF = 0.7
RCCL_LAT_US = {2: 12.0, 4: 16.0, 8: 24.0}


def allreduce_us(nbytes, n, eff=RCCL_EFF, calls=1):
    """Modelled ring exchange time of nbytes over n GPUs: `calls` latencies +
    2(n-1)/n x bytes / bus bandwidth (an all-reduce: calls 1, bytes = payload;
    the bf16 configuration's fp32 reduce-scatter + bf16 all-gather: calls 2,
    (n-1)/n x (4 + 2) B per element = 2(n-1)/n x 3 B)."""
    if n <= 1 or nbytes <= 0:
        return 0.0
    busbw = (n - 1) * XGMI_LINK_GBS * eff      # GB/s
    return calls * RCCL_LAT_US[n] + 2.0 * (n - 1) / n * nbytes / (busbw * 1e3)


def exchange_bytes(S, A, H1, H2, elt=4):
    """Bytes of each RCCL exchange of one data-parallel step (the ctx's flat
    layout: critic dWh, the critic's other tensors + stats, actor dW2, the
    actor's other tensors), as all-reduce-equivalent payload: fp32 (elt 4),
    or in the bf16 configuration an fp32 reduce-scatter + bf16 all-gather
    (elt 3: the mean of 4 and 2 B over the two collectives)."""
    ap = S * H1 + H1 + H1 * H2 + H2 + H2 * A
    cp = S * H1 + H1 + A * H1 + H1 + 2 * H1 * H2 + H2 + H2 + 1
    return {"critic_dWh": elt * 2 * H1 * H2, "critic_rest": elt * (cp - 2 * H1 * H2) + 8,
            "actor_dW2": elt * H1 * H2, "actor_rest": elt * (ap - H1 * H2),
            "calls": 2 if elt == 3 else 1}


def exposed_exchange_us(xb, win, n, eff=RCCL_EFF, small=False):
    """Exchange time on the critical path of one step.  Per network the comm
    stream runs the big call (dWh / dW2) then the tail call; `win` holds the
    measured windows from issuing each call to the join that Adam waits on
    (critic / critic_tail, actor / actor_tail): the big call starts at 0, the
    tail is issued at W - W_tail and starts when both it is issued and the big
    call is done; what runs past the join is exposed.  small: the small-batch
    path's two calls (one per network, nothing to overlap)."""
    k = xb.get("calls", 1)
    if small:
        return (allreduce_us(xb["critic_dWh"] + xb["critic_rest"], n, eff, k) +
                allreduce_us(xb["actor_dW2"] + xb["actor_rest"], n, eff, k))
    t = 0.0
    for net, big, rest in (("critic", "critic_dWh", "critic_rest"),
                           ("actor", "actor_dW2", "actor_rest")):
        w, wt = win.get(net, 0.0), win.get(net + "_tail", 0.0)
        tail_start = max(w - wt, allreduce_us(xb[big], n, eff, k))
        t += max(0.0, tail_start + allreduce_us(xb[rest], n, eff, k) - w)
    return t


def per_rank_step(cfg_name, device, n, mode, rb, dtype, steps=30, warmup=5, prof_steps=5):
    """One GPU runs rank 0's workload of an n-GPU run (bench.py --per-rank-of):
    per-rank batch B/n (strong) or B (weak), global draw of the full batch,
    the proxy communicator (every RCCL call site, the same graph-captured
    issue).  Returns the measured step and the exchange-overlap windows."""
    B0 = CONFIGS[cfg_name][4]
    b = B0 // n if mode == "strong" else B0
    sess, _, fl, _ = build_learner(cfg_name, device, 0, n, 0, dtype=dtype, per_gpu_b=b, rb=rb,
                                   proxy=True)
    el = timed(fl, sess, steps, warmup, 1)
    graphed, eager, failed = fl.step_counts()   # the timed steps: graph replays?
    rows, _ = kernel_profile(fl, sess, prof_steps)
    sess.close()
    win = {k.split("|", 1)[1]: 1e3 * v["ms"] / v["launches"] for k, v in rows.items()
           if k.startswith("xwin|")}
    busy = sum(v["ms"] for k, v in rows.items() if not k.startswith(("rccl", "xwin"))) / prof_steps
    by_kernel = summarize_profile(rows, prof_steps)[0]
    top = sorted(((k, v) for k, v in by_kernel.items() if not k.startswith("xwin")),
                 key=lambda kv: -kv[1]["ms"])[:8]
    return {"per_rank_batch": b, "step_ms": round(1000.0 * el / steps, 4),
            "step_mode": {"graph_replays": graphed, "eager_steps": eager,
                          "rccl_capture_failed": failed},
            "path": "small-batch kernels" if any(k.startswith("sb_") for k in rows)
                    else "large-batch GEMM path",
            "gpu_busy_ms": round(busy, 4),
            "window_us": {k: round(v, 1) for k, v in win.items()},
            "kernels_ms_per_step": {k: round(v["ms"] / prof_steps, 4) for k, v in top},
            # every call site: [avg us, launches per step]
            "launches_per_step": sum(v["launches"] for k, v in rows.items()
                                     if not k.startswith(("rccl", "xwin"))) / prof_steps,
            "kernels_by_phase": {k: [round(1e3 * v["ms"] / v["launches"], 2),
                                     v["launches"] / prof_steps]
                                 for k, v in sorted(rows.items(), key=lambda kv: -kv[1]["ms"])
                                 if not k.startswith("xwin")}}


def projected_scaling(cfg_name, device, rb, dtype, base_value, ns=(2, 4, 8)):
    """Projected N-GPU throughput from one GPU: the measured per-rank step
    (rank 0's exact workload via the proxy communicator) + the modelled
    exchange exposed beyond the measured overlap windows.  base_value = the
    measured 1-GPU updates/s (no communicator)."""
    S, A, H1, H2 = CONFIGS[cfg_name][:4]
    xb = exchange_bytes(S, A, H1, H2, 3 if dtype == "bf16" else 4)
    out = {"value_kind": "projected: measured per-rank step + modelled exchange "
                         "(model inputs below are assumptions; N >= 2 unmeasured on hardware)",
           "model": {"xgmi_link_GBs_per_direction": XGMI_LINK_GBS, "rccl_bus_efficiency": RCCL_EFF,
                     "rccl_latency_us": RCCL_LAT_US, "exchange_bytes": xb,
                     "formula": "step(N) = measured per-rank step (proxy communicator, graph) "
                                "+ per network, the part of its two calls (big, then tail, "
                                "serialised on the comm stream) that runs past the join, from "
                                "the measured issue-to-join windows (small-batch path: its 2 "
                                "calls, fully exposed); "
                                "T_ar = lat + 2(N-1)/N bytes / ((N-1) link eff); "
                                "pessimistic: eff halved"},
           "measured_1gpu_updates_s": base_value}
    for mode in ("strong", "weak"):
        rows = {}
        for n in ns:
            m = per_rank_step(cfg_name, device, n, mode, rb, dtype)
            small = m["path"] == "small-batch kernels"
            ex = exposed_exchange_us(xb, m["window_us"], n, small=small)
            ex_p = exposed_exchange_us(xb, m["window_us"], n, RCCL_EFF / 2, small=small)
            step = m["step_ms"] + ex / 1000.0
            step_p = m["step_ms"] + ex_p / 1000.0
            # strong: global updates/s; weak: batch-B updates processed by all ranks / s
            val = (1.0 if mode == "strong" else n) * 1000.0 / step
            val_p = (1.0 if mode == "strong" else n) * 1000.0 / step_p
            m.update({"exposed_exchange_us": round(ex, 1), "projected_step_ms": round(step, 4),
                      "projected_updates_s": round(val, 1),
                      "speedup_vs_1gpu": round(val / base_value, 3),
                      "pessimistic_speedup": round(val_p / base_value, 3)})
            rows[str(n)] = m
            log("[bench] projection %s %s N=%d: per-rank %.3f ms + exposed %.0f us -> x%.2f"
                % (cfg_name, mode, n, m["step_ms"], ex, val / base_value))
        out[mode] = rows
    return out


def timed(fl, sess, steps, warmup, world):
    import torch
    import torch.distributed as dist
    for _ in range(warmup):
        fl.step()
    sess.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    sess.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fl.step()
    sess.sync()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    el = t1 - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


def kernel_profile(fl, sess, steps):
    from distributed_ddpg_amd.learner import Profile
    prof = Profile(sess)
    prof.enable(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        fl.step()
    sess.sync()
    wall = time.perf_counter() - t0
    rows = prof.read()
    prof.enable(False)
    return rows, wall


# A pack launch runs the same kernel body as the single launch over up to
# GH_MAXP independent GEMMs (csrc/gemm_h3.h, gemm_h3m.h): the roofline rates
# that body, so its pack launches count with it (launches, FLOP, time added;
# the members and their launches per step are listed in the record).
BODY_OF = {"gemm_h3m_pack_kernel<RK,KR,NP=3>": "gemm_h3m_kernel<RK,KR,NP=3>",
           "gemm_h16i_pack_kernel<RK,KR,NP=1>": "gemm_h16i_kernel<RK,KR,NP=1>"}


def summarize_profile(rows, steps):
    by_kernel = {}
    for key, r in rows.items():
        sym = key.split("|")[0]
        k = by_kernel.setdefault(sym, {"ms": 0.0, "launches": 0, "flops": 0.0, "bytes": 0.0})
        for f in ("ms", "launches", "flops", "bytes"):
            k[f] += r[f]
    bodies = {}
    for sym, r in by_kernel.items():
        k = bodies.setdefault(BODY_OF.get(sym, sym), {"ms": 0.0, "launches": 0, "flops": 0.0,
                                                      "bytes": 0.0, "members": {}})
        for f in ("ms", "launches", "flops", "bytes"):
            k[f] += r[f]
        k["members"][sym] = r["launches"] / steps
    # the collectives' events run on the comm stream concurrently with kernels,
    # and the xwin records are exchange-overlap windows (spans of the step):
    # neither is GPU-busy time nor a roofline candidate
    side = ("rccl", "xwin")
    comp = {k: v for k, v in bodies.items() if not k.startswith(side)}
    gpu_ms = sum(r["ms"] for k, r in rows.items() if not k.startswith(side)) / steps
    gemm_ms = sum(r["ms"] for k, r in comp.items() if k.startswith("gemm")) / steps
    gemm_flops = sum(r["flops"] for k, r in comp.items() if k.startswith("gemm")) / steps
    dom = max(comp.items(), key=lambda kv: kv[1]["ms"])
    return by_kernel, dom, gpu_ms, gemm_ms, gemm_flops


def action_selection_latency(actor, S, calls=2000):
    """actor.predict on one state (ddpg.py:68-70), host wall time per call
    including the device round trip (states in, action out)."""
    s = np.random.default_rng(0).standard_normal((1, S)).astype(np.float32)
    for _ in range(50):
        actor.predict(s)
    t0 = time.perf_counter()
    for _ in range(calls):
        actor.predict(s)
    el = time.perf_counter() - t0
    return {"batch": 1, "us_per_call": round(1e6 * el / calls, 2), "calls": calls}


def worker_env_step_latency(fl, rb, actor, S, n=1000):
    """The reference worker's device work per env step (ddpg.py:68-113 with
    the fused learner): actor.predict on one state, ReplayBuffer.add of one
    transition, learner.step with stats -- host wall time per env step."""
    st = np.random.default_rng(1).standard_normal((n + 101, S)).astype(np.float32)
    ts = []
    for i in range(n + 100):
        t0 = time.perf_counter()
        a = actor.predict(st[i:i + 1])
        rb.add(st[i], a[0], 0.5, False, st[i + 1])
        fl.step(stats=True)
        ts.append(1e6 * (time.perf_counter() - t0))
    p10, p50, p90 = np.percentile(ts[100:], [10, 50, 90])
    return {"n": n, "p10_us": round(float(p10), 1), "median_us": round(float(p50), 1),
            "p90_us": round(float(p90), 1)}


def pmc_traffic(cfg_name, kernel, launches_per_step):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (profiles/*_pmc_<config>.json, written by profiles/pmc_traffic.py from a
    FETCH_SIZE pass and a WRITE_SIZE pass of this same bench command, with the
    gfx950 FETCH_SIZE x2 correction).  PMC counters cannot be read in-process."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_%s.json" % cfg_name)))
    for fn in reversed(files):
        try:
            k = json.load(open(fn))["kernels"].get(kernel)
        except (OSError, ValueError):
            continue
        if not k:
            continue
        # the PMC pass must have profiled the same launch set as this run
        lps = k.get("launches_per_step")
        if lps is None or abs(lps - launches_per_step) > 1e-6:
            return None, "%s: launches/step %s != %s (stale pass, not used)" % (
                os.path.relpath(fn, ROOT), lps, launches_per_step)
        return round(k["traffic_bytes_per_launch"]), os.path.relpath(fn, ROOT)
    return None, None


def body_traffic(cfg_name, dom):
    """pmc_traffic of a kernel body: the launch-weighted mean over its members
    (single and pack launches), each checked against its launches per step."""
    tot, n, srcs = 0.0, 0.0, []
    for sym, lps in dom["members"].items():
        t, src = pmc_traffic(cfg_name, sym, lps)
        if t is None:
            return None, src
        tot += t * lps
        n += lps
        srcs.append(src)
    return (round(tot / n) if n else None), ", ".join(sorted(set(srcs)))


def kernel_peak(name):
    """MFMA peak a kernel is rated against: bf16 operands (NP=1 twins, the
    256 x 256 bf16 kernel) 2.5 PF; fp32 on the bf16 pipe (three-plane twins /
    gemm_s3, six products per MAC) 2.5 PF / 6; the fp32-input MFMA 157.3 TF."""
    if name.startswith("gemm_h256") or (name.startswith(("gemm_h", "gemm_s3")) and "NP=1" in name):
        return PEAK_BF16_MFMA_TFLOPS
    if name.startswith(("gemm_h", "gemm_s3")):
        return PEAK_S3_FP32EQ_TFLOPS
    return PEAK_FP32_MFMA_TFLOPS


def mfma_busy_step(cfg_name, step_ms):
    """Counter-measured MFMA busy of the whole step from the newest committed
    PMC pass (profiles/**/*mfma_<config>.json, SQ_VALU_MFMA_BUSY_CYCLES per
    launch x launches per step): busy cycles / (1024 SIMDs x step time x
    2.4 GHz) -- at the peak clock, so a lower bound of the busy fraction at
    the clock the chip held.  None when no pass is committed."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "*mfma_%s.json" % cfg_name),
                             recursive=True))   # profiles/rN/...: newest round last
    for fn in reversed(files):
        try:
            ks = json.load(open(fn))["kernels"]
        except (OSError, ValueError, KeyError):
            continue
        cyc = sum(k["mfma_busy_cycles_per_launch"] * k["launches_per_step"] for k in ks.values())
        return {"busy_at_2.4GHz": round(cyc / (1024 * step_ms * 1e-3 * 2.4e9), 4),
                "source": os.path.relpath(fn, ROOT)}
    return None


def _cpu_model():
    cpu, cores = "unknown", os.cpu_count()
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        kv = dict(l.split(":", 1) for l in out.splitlines() if ":" in l)
        cpu = kv.get("Model name", cpu).strip()
        cores = int(kv["Core(s) per socket"]) * int(kv.get("Socket(s)", "1"))
    except Exception:
        pass
    return cpu, cores


def _ref_replay(cfg_name, rows_n):
    """The reference's deque replay (oracle/torch_cpu.py DequeReplay,
    replay_buffer.py:12-47) filled with rows_n synthetic transitions."""
    from oracle.torch_cpu import DequeReplay
    S, A, _, _, _, scale, _ = CONFIGS[cfg_name]
    rng = np.random.default_rng(0)
    rb = DequeReplay(rows_n, seed=1234)
    chunk = 100_000
    for lo in range(0, rows_n, chunk):
        m = min(chunk, rows_n - lo)
        rb.fill(rng.standard_normal((m, S)), (rng.uniform(-1, 1, (m, A)) * scale).astype(np.float32),
                rng.standard_normal(m), rng.random(m) < 0.01, rng.standard_normal((m, S)))
    return rb


def _cpu_leg(cfg_name, threads, budget_s, rb, max_steps=200):
    """Time the reference's learner step on the CPU: replay_buffer.sample_batch
    over a full deque (DequeReplay) + the torch-CPU restatement of the eight
    sess.run calls (oracle/torch_cpu.py) at `threads` intra-op threads, bounded
    by budget_s seconds or max_steps steps (whichever first, >= 1 step)."""
    import torch
    from oracle.torch_cpu import TorchCPULearner
    S, A, H1, H2, B, scale, _ = CONFIGS[cfg_name]
    torch.set_num_threads(threads)
    L = TorchCPULearner(S, A, H1, H2, scale, seed=1)
    L.step(*rb.sample_batch(B))  # warm-up
    n, t_sample, t0 = 0, 0.0, time.perf_counter()
    while True:
        ts = time.perf_counter()
        batch = rb.sample_batch(B)
        t_sample += time.perf_counter() - ts
        L.step(*batch)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= max_steps:
            break
    return {"value": round(n / el, 3), "unit": "updates/s", "threads": threads, "steps": n,
            "seconds": round(el, 2), "sample_batch_ms": round(1e3 * t_sample / n, 3)}


def cpu_baseline(cfg_name, threads):
    """the reference's TF CPU path cannot run on the GPU box, so
    the baseline is the reference's own host replay sampling (deque +
    random.sample + np.array stacking over a full 1e6-row buffer) plus a
    torch-CPU eager, op-for-op restatement of its eight sess.run calls per
    learner step, timed on this host at `threads` threads (the box's CPU
    share), at 1 thread and at os.cpu_count() threads; at the bench config, at
    C2 (B=64) and at C1 (BASELINE configs[0]: MountainCar-shaped 400/300,
    B=64)."""
    import torch
    cpu, cores = _cpu_model()
    allc = os.cpu_count() or 1
    prev = torch.get_num_threads()
    t0 = time.perf_counter()
    rb = _ref_replay(cfg_name, REPLAY_ROWS)
    fill_s = time.perf_counter() - t0
    main = _cpu_leg(cfg_name, threads, 12.0, rb)
    one = _cpu_leg(cfg_name, 1, 8.0, rb)
    del rb
    out = {}
    for name in ("c2", "c1"):
        rbs = _ref_replay(name, REPLAY_ROWS)
        out[name + "_b64"] = _cpu_leg(name, threads, 3.0, rbs, 2000)
        out[name + "_b64_one_thread"] = _cpu_leg(name, 1, 3.0, rbs, 2000)
        if name == "c2" and allc != threads:
            # os.cpu_count() threads: the box's cgroup share is 16 CPUs, so this
            # oversubscribes; at C3 one step took 36 s this way (round 3), so
            # the all-CPU figure is reported at C2 only
            out["c2_b64_all_cpus"] = _cpu_leg(name, allc, 3.0, rbs, 2000)
        del rbs
    torch.set_num_threads(prev)
    res = {"value": main["value"], "unit": "updates/s", "cores": threads, "kind": "port",
           "sample": "%d learner steps of %s in %.1fs, each = the reference's sample_batch over "
                     "a full %d-row deque (%.1f ms of it) + a torch-CPU fp32 eager restatement of "
                     "its 8 sess.run calls (oracle/torch_cpu.py; TF 1.3 is not installable on the "
                     "box), %d threads on %s (%d physical cores on the host, os.cpu_count() = %d; "
                     "the GPU box's CPU share is 16 threads)"
                     % (main["steps"], cfg_name.upper(), main["seconds"], REPLAY_ROWS,
                        main["sample_batch_ms"], threads, cpu, cores, allc),
           "one_thread": one, "deque_fill_s": round(fill_s, 1),
           "cpu_model": cpu, "host_cores": cores, "os_cpu_count": allc,
           "historical_reference": "about 52 updates/s end to end incl. env + gRPC "
                                   "(BASELINE.md, 2017 TF CPU; context only)"}
    res.update(out)
    return res


def step_latency_percentiles(fl, sess, n):
    """Per-step wall time with a host sync after every step (latency view; the
    headline value above keeps the steps pipelined)."""
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fl.step()
        sess.sync()
        ts.append(1000.0 * (time.perf_counter() - t0))
    p10, p50, p90 = np.percentile(ts, [10, 50, 90])
    return {"n": n, "p10_ms": round(float(p10), 4), "median_ms": round(float(p50), 4),
            "p90_ms": round(float(p90), 4)}


# ---------------------------------------------------------------- the contract line
# The driver parses the ONE stdout line; a 26.8 KB line came back unparsed in
# round 5 (a 14.5 KB one parsed in round 4).  The full record (per-call-site
# kernel tables, per-rank projections) goes to the detail file / stderr; the
# stdout line carries the contract fields, roofline, cpu_baseline and compact
# summaries, and is held under CONTRACT_LINE_MAX bytes.
CONTRACT_LINE_MAX = 8192
CONTRACT_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                 "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                 "roofline", "cpu_baseline")


def _top_kernels(kernels, n):
    """{name: [avg_us, launches per step]} of the n kernels with the most time."""
    rows = sorted(kernels.items(), key=lambda kv: -kv[1].get("ms_per_step",
                                                             kv[1]["avg_us"] * kv[1]["per_step"]))
    return {k: [v["avg_us"], v["per_step"]] for k, v in rows[:n]}


def _compact_projection(pr):
    """Per mode and N: per-rank batch and step, exposed exchange, speedup
    (pessimistic beside it), step mode as 'graph replays/eager steps'."""
    if not pr:
        return pr
    out = {"value_kind": "projected (measured per-rank step + modelled exchange; N>=2 "
                         "unmeasured on hardware)",
           "model": {"link_GBs": pr["model"]["xgmi_link_GBs_per_direction"],
                     "eff": pr["model"]["rccl_bus_efficiency"],
                     "lat_us": pr["model"]["rccl_latency_us"]},
           "measured_1gpu_updates_s": pr.get("measured_1gpu_updates_s")}
    for mode in ("weak", "strong"):
        if mode not in pr:
            continue
        out[mode] = {}
        for n, m in pr[mode].items():
            sm = m.get("step_mode") or {}
            out[mode][n] = {"b": m["per_rank_batch"], "step_ms": m["step_ms"],
                            "exposed_exchange_us": m["exposed_exchange_us"],
                            "speedup": m["speedup_vs_1gpu"], "pess": m["pessimistic_speedup"],
                            "step_mode": "%s/%s%s" % (sm.get("graph_replays"),
                                                      sm.get("eager_steps"),
                                                      "/capture-failed"
                                                      if sm.get("rccl_capture_failed") else "")}
    return out


def _compact_cpu(cb):
    if not cb:
        return cb
    keep = ("value", "unit", "cores", "kind", "sample", "cpu_model", "host_cores",
            "os_cpu_count", "historical_reference")
    out = {k: cb[k] for k in keep if k in cb}
    for k, v in cb.items():
        if isinstance(v, dict) and "value" in v:   # one_thread, c2_b64, c1_b64, ...
            out[k] = {"value": v["value"], "threads": v.get("threads")}
    return out


def compact_line(full, limit=CONTRACT_LINE_MAX):
    """The stdout contract line built from the full record: every contract
    key, the full roofline and cpu_baseline, compact c5_bf16 / small_batch /
    projected_scaling summaries.  Optional blocks are dropped (in a fixed
    order, named in `dropped`) until the line fits `limit` bytes."""
    out = {k: full[k] for k in full
           if k not in ("kernels", "kernels_by_phase", "projected_scaling", "small_batch",
                        "c5_bf16", "cpu_baseline")}
    out["cpu_baseline"] = _compact_cpu(full.get("cpu_baseline"))
    if "kernels" in full:
        out["kernels"] = _top_kernels(full["kernels"], 10)
    if full.get("projected_scaling"):
        out["projected_scaling"] = _compact_projection(full["projected_scaling"])
    sb = full.get("small_batch")
    if sb:
        out["small_batch"] = {k: sb[k] for k in ("value", "ms_per_step", "step_latency",
                                                 "kernels_per_step", "gpu_busy_ms_per_step",
                                                 "launch_overhead_us_per_step",
                                                 "action_selection", "worker_env_step")
                             if k in sb}
        b2 = sb.get("b256")
        if b2:
            dp = b2.get("dp_rank0_of_8_weak") or {}
            out["small_batch"]["b256"] = {
                "value": b2["value"], "ms_per_step": b2["ms_per_step"],
                "sync_median_ms": b2["step_latency"]["median_ms"], "path": b2["path"],
                "kernels_per_step": b2["kernels_per_step"],
                "dp_rank0_of_8_weak_step_ms": dp.get("step_ms")}
    c5 = full.get("c5_bf16")
    if c5:
        out["c5_bf16"] = {k: v for k, v in c5.items() if k not in ("kernels", "projected_scaling")}
        if "kernels" in c5:
            out["c5_bf16"]["kernels"] = _top_kernels(c5["kernels"], 6)
        if c5.get("projected_scaling"):
            out["c5_bf16"]["projected_scaling"] = _compact_projection(c5["projected_scaling"])
    dropped = []
    for path in (("c5_bf16", "kernels"), ("kernels",), ("small_batch", "b256"),
                 ("cpu_baseline", "historical_reference"), ("c5_bf16", "projected_scaling"),
                 ("projected_scaling",), ("small_batch",), ("c5_bf16",)):
        if len(json.dumps(out)) <= limit:
            break
        d = out
        for p in path[:-1]:
            d = d.get(p) or {}
        if path[-1] in d:
            del d[path[-1]]
            dropped.append(".".join(path))
    if dropped:
        out["dropped"] = dropped
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--replay", type=int, default=REPLAY_ROWS)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-small", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=20)
    ap.add_argument("--dtype", default=None, choices=["fp32", "bf16"],
                    help="GEMM operand precision (default: fp32, bf16 for c5)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: per-GPU batch fixed at the config's B; strong: global batch "
                         "fixed at B (B/N rows per GPU)")
    ap.add_argument("--per-rank-of", type=int, default=0, metavar="N",
                    help="on ONE GPU, time exactly rank 0's workload of an N-GPU run (per-rank "
                         "batch per --scaling, proxy communicator) and print its projection")
    ap.add_argument("--no-project", action="store_true",
                    help="skip the projected_scaling block (N=1 default runs only)")
    ap.add_argument("--detail", default=None, metavar="PATH",
                    help="where the full JSON record goes (default gpurun_out/bench_detail.json); "
                         "stdout carries the compact contract line")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start the N ranks here, before this process touches the GPU
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("[bench] note: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))
    import torch
    if os.environ.get("DDPG_BENCH_ONE_DEVICE") == "1":
        # rehearsal of an N-rank run on a one-GPU box (every rank on device 0,
        # with DDPG_LIB_PATH=tools/shm/libddpg_shm.so standing in for RCCL,
        # which refuses two ranks on one device; tools/gpu/r6_rehearse.sh)
        local = 0
    if local >= torch.cuda.device_count():
        raise SystemExit("[bench] rank %d: LOCAL_RANK %d but only %d GPU(s) visible"
                         % (rank, local, torch.cuda.device_count()))
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        with stdout_to_stderr():   # Gloo prints its peer-connection line on fd 1
            dist.init_process_group("gloo", rank=rank, world_size=world)

    cfg = args.config
    dtype = args.dtype or DEFAULT_DTYPE[cfg]
    S, A, H1, H2, B0, scale, label = CONFIGS[cfg]
    if args.per_rank_of > 1:
        if world != 1:
            raise SystemExit("[bench] --per-rank-of runs on one GPU")
        n = args.per_rank_of
        sess1, rb1, fl1, _ = build_learner(cfg, local, 0, 1, args.replay, dtype=dtype)
        base = args.steps / timed(fl1, sess1, args.steps, args.warmup, 1)
        sess1.close()
        pr = projected_scaling(cfg, local, rb1, dtype, round(base, 3), ns=(n,))
        print(json.dumps({"metric": "projected actor+critic updates/sec on %d GPUs (%s scaling, "
                                    "rank 0's workload measured on one GPU)" % (n, args.scaling),
                          "value": pr[args.scaling][str(n)]["projected_updates_s"],
                          "value_kind": "projected", "measured_on_n_gpus": 1,
                          "unit": "updates/s", "n_gpus": 1, "per_rank_of": n,
                          "scaling": args.scaling, "dtype": dtype, "config": {"workload": label},
                          "projected_scaling": _compact_projection(pr)}), flush=True)
        log("[bench] per-rank detail: " + json.dumps(pr))
        return
    strong = args.scaling == "strong"
    if strong and B0 % world:
        raise SystemExit("[bench] strong scaling: batch %d not divisible by %d GPUs" % (B0, world))
    B = B0 // world if strong else B0   # rows per GPU
    if strong:
        label = label.replace("batch %d/GPU" % B0, "global batch %d (%d/GPU)" % (B0, B))
    label = "%s, %s GEMM operands (fp32 master weights/accumulation)" % (label, dtype)
    sess, rb, fl, _ = build_learner(cfg, local, rank, world, args.replay, dtype=dtype, per_gpu_b=B)
    el = timed(fl, sess, args.steps, args.warmup, world)
    ms = 1000.0 * el / args.steps
    # weak: batch-B updates processed by all ranks per second; strong: global updates per second
    value = (1 if strong else world) * args.steps / el

    lat = step_latency_percentiles(fl, sess, min(100, max(10, args.steps)))
    rows, _ = kernel_profile(fl, sess, args.profile_steps)
    by_kernel, (dom_name, dom), gpu_ms, gemm_ms, gemm_flops = summarize_profile(
        rows, args.profile_steps)
    from distributed_ddpg_amd.flops import flops_per_step
    step_flops = flops_per_step(S, A, H1, H2, B)   # per GPU
    dom_avg_ms = dom["ms"] / dom["launches"]
    dom_flops = dom["flops"] / dom["launches"]
    achieved = dom_flops / (dom_avg_ms * 1e-3) / 1e12
    peak = kernel_peak(dom_name)
    # the pipe the step's GEMMs run on: bf16 operands at 2.5 PF; fp32 contexts
    # on the same bf16 pipe at six plane products per MAC (2.5 PF / 6)
    step_peak = PEAK_BF16_MFMA_TFLOPS if dtype == "bf16" else PEAK_S3_FP32EQ_TFLOPS
    traffic, traffic_src = (body_traffic(cfg, dom)
                            if world == 1 else (None, "PMC passes are single-GPU"))
    roofline = {"bound": "mfma", "kernel": dom_name, "achieved": round(achieved, 2),
                "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": traffic,
                "frac_vs_fp32_mfma_peak": round(achieved / PEAK_FP32_MFMA_TFLOPS, 4),
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": dom["bytes"] / dom["launches"],
                "avg_launch_us": round(dom_avg_ms * 1e3, 2),
                "flop_per_launch": dom_flops, "launches_per_step":
                    dom["launches"] / args.profile_steps, "launches": dom["members"]}
    metric = ("actor+critic updates/sec (global batch %d, %d-wide MLPs)" % (B0, H1) if strong else
              "actor+critic updates/sec (batch %d per GPU, %d-wide MLPs)" % (B, H1))
    out = {
        "metric": metric,
        "value": round(value, 3), "unit": "updates/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
        "scaling": args.scaling, "vs_baseline": None, "dtype": dtype,
        "data": "synthetic (replay ring of %d N(0,1)/U(-1,1)/Bernoulli(0.01) transitions; "
                "random-init weights)" % args.replay,
        "config": {"workload": label, "state_dim": S, "action_dim": A, "hidden": [H1, H2],
                   "global_batch": B * world, "per_gpu_batch": B,
                   "parallelism": "dp%d" % world},
        "samples_per_s": round(world * args.steps / el * B, 1),
        # whole-step algorithmic FLOP rate against the pipe the GEMMs use
        # (step_peak); the fp32-peak reading beside it; the counter-measured
        # MFMA busy of the step from the committed PMC pass
        "mfma_util_step": round(step_flops / (ms * 1e-3) / 1e12 / step_peak, 4),
        "mfma_util_step_peak_tflops": step_peak,
        "step_frac_vs_fp32_mfma_peak": round(step_flops / (ms * 1e-3) / 1e12
                                             / PEAK_FP32_MFMA_TFLOPS, 4),
        "mfma_busy_step_counter": mfma_busy_step(cfg, ms) if world == 1 else None,
        "step_tflops": round(step_flops / (ms * 1e-3) / 1e12, 2),
        "gemm_tflops": round(gemm_flops / (gemm_ms * 1e-3) / 1e12, 2) if gemm_ms else None,
        "gpu_busy_ms_per_step": round(gpu_ms, 4),
        "step_latency": lat,
        "roofline": roofline,
        "kernels": {k: {"avg_us": round(1e3 * v["ms"] / v["launches"], 2),
                        "per_step": v["launches"] / args.profile_steps,
                        "ms_per_step": round(v["ms"] / args.profile_steps, 4)}
                    for k, v in sorted(by_kernel.items(), key=lambda kv: -kv[1]["ms"])},
        # the same launches split by call site ("<kernel>|<phase>")
        "kernels_by_phase": {k: {"avg_us": round(1e3 * v["ms"] / v["launches"], 2),
                                 "per_step": v["launches"] / args.profile_steps}
                             for k, v in sorted(rows.items(), key=lambda kv: -kv[1]["ms"])},
    }
    if world > 1:
        # the data-parallel exchange (rank 0's comm-stream events: these
        # include waiting for the slowest rank); step_flops above are per GPU
        out["exchange"] = {k: {"avg_us": round(1e3 * v["ms"] / v["launches"], 2),
                               "per_step": v["launches"] / args.profile_steps,
                               "MB_per_step": round(v["bytes"] / args.profile_steps / 1e6, 3)}
                           for k, v in by_kernel.items() if k.startswith("rccl")}
    hbm = {}
    for key in ("adam+reduce+soft_update", "adam+soft_update", "adam", "soft_update", "gather"):
        if key in by_kernel and by_kernel[key]["ms"] > 0:
            k = by_kernel[key]
            hbm[key] = round(k["bytes"] / (k["ms"] * 1e-3) / 1e9, 1)
    out["hbm_GBs"] = hbm
    if world == 1 and rank == 0 and cfg in ("c3", "c5") and not args.no_project:
        # SURVEY §7 / BASELINE: >= 6x at 8 GPUs -- rank 0's exact per-rank
        # workload measured here (strong and weak), the exchange modelled
        out["projected_scaling"] = projected_scaling(cfg, local, rb, dtype, round(value, 3))

    if world == 1 and rank == 0 and not args.no_small and cfg != "c2":
        s2, rb2, fl2, actor2 = build_learner("c2", local, 0, 1, REPLAY_ROWS)
        el2 = timed(fl2, s2, 500, 50, 1)
        # the reference's worker synchronises every env step (action
        # selection reads the updated actor, ddpg.py:68-70,86-113): the
        # synchronous per-step latency is what its caller sees
        lat2 = step_latency_percentiles(fl2, s2, 300)
        rows2, wall2 = kernel_profile(fl2, s2, 100)
        busy2 = sum(r["ms"] for r in rows2.values()) / 100
        nk2 = sum(r["launches"] for r in rows2.values()) / 100
        out["small_batch"] = {
            "workload": CONFIGS["c2"][6], "value": round(500 / el2, 1), "unit": "updates/s",
            "ms_per_step": round(1000 * el2 / 500, 4),
            "step_latency": lat2,
            "kernels_per_step": nk2, "gpu_busy_ms_per_step": round(busy2, 4),
            "launch_overhead_us_per_step": round(1000 * (1000 * el2 / 500 - busy2), 1),
            "action_selection": action_selection_latency(actor2, CONFIGS["c2"][0]),
            "worker_env_step": worker_env_step_latency(fl2, rb2, actor2, CONFIGS["c2"][0])}
        s2.close()
        # the reference's default batch (B = 256): one GPU, and rank 0 of an
        # 8-rank data-parallel run at that per-rank batch (weak: the
        # reference's workers each train on their own 256 rows)
        s2b, _, fl2b, _ = build_learner("c2b", local, 0, 1, 0, rb=rb2)
        el2b = timed(fl2b, s2b, 300, 30, 1)
        lat2b = step_latency_percentiles(fl2b, s2b, 200)
        rows2b, _ = kernel_profile(fl2b, s2b, 50)
        s2b.close()
        dp2b = per_rank_step("c2b", local, 8, "weak", rb2, "fp32")
        out["small_batch"]["b256"] = {
            "workload": CONFIGS["c2b"][6], "value": round(300 / el2b, 1), "unit": "updates/s",
            "ms_per_step": round(1000 * el2b / 300, 4), "step_latency": lat2b,
            "path": "small-batch kernels" if any(k.startswith("sb_") for k in rows2b)
                    else "large-batch GEMM path",
            "kernels_per_step": sum(r["launches"] for r in rows2b.values()) / 50,
            "gpu_busy_ms_per_step": round(sum(r["ms"] for r in rows2b.values()) / 50, 4),
            "dp_rank0_of_8_weak": dict(dp2b, note="rank 0's step of an 8-rank data-parallel "
                                       "run at 256 rows per rank, measured through the 1-rank "
                                       "proxy communicator (RCCL calls as identities: the "
                                       "8-rank exchange itself is not included)")}
    if not args.no_small and cfg == "c3":
        # BASELINE configs[4] (C5, bf16) as a secondary line on every rank: same
        # step, same accounting and scaling mode, its own dominant kernel
        sess.close()
        S5, A5, H15, H25, B50, _, label5 = CONFIGS["c5"]
        B5 = B50 // world if strong else B50
        s5, rb5, fl5, _ = build_learner("c5", local, rank, world, args.replay, dtype="bf16",
                                        per_gpu_b=B5)
        el5 = timed(fl5, s5, 30, 5, world)
        rows5, _ = kernel_profile(fl5, s5, 10)
        bk5, (dn5, d5), gpu5, _, _ = summarize_profile(rows5, 10)
        f5 = flops_per_step(S5, A5, H15, H25, B5)
        ms5 = 1000.0 * el5 / 30
        ach5 = (d5["flops"] / d5["launches"]) / (d5["ms"] / d5["launches"] * 1e-3) / 1e12
        pk5 = kernel_peak(dn5)
        tr5, tr5_src = body_traffic("c5", d5) if world == 1 else (None, None)
        out["c5_bf16"] = {
            "workload": label5 + ", bf16 GEMM operands (fp32 master weights/accumulation)",
            "value": round((1 if strong else world) * 30 / el5, 3), "unit": "updates/s",
            "n_gpus": world, "per_gpu_batch": B5, "scaling": args.scaling,
            "ms_per_step": round(ms5, 4),
            "dtype": "bf16", "gpu_busy_ms_per_step": round(gpu5, 4),
            "step_tflops": round(f5 / (ms5 * 1e-3) / 1e12, 2),
            "mfma_util_step": round(f5 / (ms5 * 1e-3) / 1e12 / PEAK_BF16_MFMA_TFLOPS, 4),
            "mfma_busy_step_counter": mfma_busy_step("c5", ms5) if world == 1 else None,
            "roofline": {"bound": "mfma", "kernel": dn5, "achieved": round(ach5, 2), "peak": pk5,
                         "unit": "TFLOP/s", "frac": round(ach5 / pk5, 4), "traffic": tr5,
                         "traffic_source": tr5_src,
                         "avg_launch_us": round(1e3 * d5["ms"] / d5["launches"], 2),
                         "launches_per_step": d5["launches"] / 10, "launches": d5["members"]},
            "kernels": {k: {"avg_us": round(1e3 * v["ms"] / v["launches"], 2),
                            "per_step": v["launches"] / 10}
                        for k, v in sorted(bk5.items(), key=lambda kv: -kv[1]["ms"])}}
        if world == 1 and not args.no_project:
            out["c5_bf16"]["projected_scaling"] = projected_scaling(
                "c5", local, rb5, "bf16", out["c5_bf16"]["value"])
        s5.close()
        sess = None
    if world == 1 and rank == 0 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(cfg, min(16, os.cpu_count() or 1))
    else:
        out["cpu_baseline"] = None
    if rank == 0:
        # full record: detail file + stderr; stdout: the compact contract line
        detail = args.detail or os.path.join(ROOT, "gpurun_out", "bench_detail.json")
        try:
            os.makedirs(os.path.dirname(detail), exist_ok=True)
            with open(detail, "w") as f:
                json.dump(out, f)
            log("[bench] full record: %s" % detail)
        except OSError as e:
            log("[bench] detail file not written (%s)" % e)
        print(json.dumps(compact_line(out)), flush=True)
    if sess is not None:
        sess.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
