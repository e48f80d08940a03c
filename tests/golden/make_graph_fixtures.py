"""Golden learner trajectories produced by EXECUTING the reference's own TF graph.

Run ONLY in the build container (reads /root/reference):
    python tests/golden/make_graph_fixtures.py

The reference's InvertedPendulum MetaGraphDef (`model_ddpg/model-1410.meta`,
TF 1.3) is run by tfgraph.py's interpreter, in float64, from the reference's
own checkpoint `model-1410` (weights, target weights, Adam m/v slots and beta
powers: a resumed run with non-trivial bias correction).  Each learner step
issues exactly the session calls of ddpg.py:86-113:

    target_q = critic.predict_target(s2, actor.predict_target(s2))   :90
    y        = r if t else r + gamma * target_q                     :92-97
    q, _, L  = critic.train(s, a, y)          [out, optimize, loss]  :100
    a_outs   = actor.predict(s)                                      :106
    grads    = critic.action_gradients(s, a_outs)                    :107
    actor.train(s, grads[0])                                         :109
    actor.update_target_network(); critic.update_target_network()    :112-113

i.e. the graph nodes: Mul_1 (actor target out), FullyConnected_13/BiasAdd
(critic target out), [FullyConnected_9/BiasAdd, Adam_1, MeanSquare/Mean],
Mul (actor out), gradients_2/FullyConnected_7/MatMul_grad/MatMul (dQ/da, grad_ys
= ones), Adam (actor ApplyAdam x5 + beta powers, grad_ys = -a_gradient via
Neg(Placeholder)), Assign_3..7 and Assign_8..15 (soft updates).

Output graph_ip1410.npz (plain data): the initial state (Adam slots and beta
powers; weights are in ip_model1410.npz), per-step inputs (float64, as the
reference's replay returns them) and outputs, the gradients every ApplyAdam
consumed, and the full state after the last step (float32-rounded arrays;
scalars in float64).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/InvertedPendulum/model_ddpg/model-1410"
MC = "/root/reference/results/model_ddpg/model-120"
sys.path.insert(0, HERE)
import tfbundle  # noqa: E402
import tfgraph  # noqa: E402

ACTOR = ["FullyConnected/W", "FullyConnected/b", "FullyConnected_1/W", "FullyConnected_1/b",
         "FullyConnected_2/W"]
CRITIC = ["FullyConnected_%d/%s" % (i, w) for i in (6, 7, 8, 9) for w in ("W", "b")]
ACTOR_T = ["FullyConnected_3/W", "FullyConnected_3/b", "FullyConnected_4/W",
           "FullyConnected_4/b", "FullyConnected_5/W"]
CRITIC_T = ["FullyConnected_%d/%s" % (i, w) for i in (10, 11, 12, 13) for w in ("W", "b")]
POWERS = ["beta1_power", "beta2_power", "beta1_power_1", "beta2_power_1"]
GAMMA = 0.99
B, STEPS = 64, 3


def adam_grad_inputs(nodes, group):
    """The gradient tensor each ApplyAdam of `group` ('Adam' / 'Adam_1') consumes."""
    out = {}
    for name, (op, inputs, _) in nodes.items():
        if op == "ApplyAdam" and name.startswith(group + "/update_"):
            out[inputs[0]] = inputs[9]
    return out


# per graph: the actor output / target-actor output nodes (the InvertedPendulum
# graph multiplies tanh by action_scale, networks.py:61; the older MountainCar
# graph -- networks.py at the time of model-120, scale 1 -- fetches the tanh)
OUT_NODES = {"ip": ("Mul", "Mul_1"), "mc": ("FullyConnected_2/Tanh", "FullyConnected_5/Tanh")}


def fresh_optimizer(sess, nodes):
    """Run the graph's own initializers of every Adam slot and beta power
    (`<var>/Adam/Assign` <- zeros, `beta*_power*/Assign` <- 0.9 / 0.999): the
    optimizer state of a training run that starts from these weights."""
    inits = [k for k, (op, _, _) in nodes.items() if op == "Assign" and k.endswith("/Assign") and
             ("/Adam/" in k or "/Adam_1/" in k or k.startswith("beta"))]
    assert len(inits) == 2 * 13 + 4, len(inits)
    sess.run(inits)


def trajectory(meta, ckpt, graph, batch_fn, steps, fresh=False, scaler=None):
    """Execute `steps` learner steps (the session calls of ddpg.py:86-113) of the
    reference graph `meta` from checkpoint `ckpt`.  batch_fn(rng) returns one
    replay batch (s, a, r, t, s2) as the reference's replay returns it; states
    go through the scaler's (x - mean) / scale first when one is given
    (networks.py:65-69,164-168)."""
    nodes = tfgraph.read_graph(meta + ".meta")
    state = tfbundle.read_checkpoint(ckpt)
    sess = tfgraph.Session(nodes, state, dtype=np.float64)
    if fresh:
        fresh_optimizer(sess, nodes)
    g_actor = adam_grad_inputs(nodes, "Adam")
    g_critic = adam_grad_inputs(nodes, "Adam_1")
    assert sorted(g_actor) == sorted(ACTOR) and sorted(g_critic) == sorted(CRITIC)
    out, out_t = OUT_NODES[graph]
    pre = (lambda x: x) if scaler is None else (lambda x: (x - scaler[0]) / scaler[1])
    rng = np.random.default_rng(1410 if graph == "ip" else 120)
    fx = {}
    for k in POWERS:
        fx["init/" + k] = np.float64(sess.vars[k])
    for k in ACTOR + CRITIC:
        fx["init/%s/Adam" % k] = sess.vars[k + "/Adam"].astype(np.float32)
        fx["init/%s/Adam_1" % k] = sess.vars[k + "/Adam_1"].astype(np.float32)
    for step in range(steps):
        s, a, r, t, s2 = batch_fn(rng)
        ps, ps2 = pre(s), pre(s2)
        a2 = sess.run(out_t, {"InputData_1/X": ps2})
        target_q = sess.run("FullyConnected_13/BiasAdd", {"InputData_4/X": ps2,
                                                          "InputData_5/X": a2})
        # GAMMA * target_q[k] multiplies a float32 array in the reference: the
        # Python-float gamma enters as float32 (ddpg.py:97)
        y = np.where(t[:, None], r[:, None], r[:, None] + np.float64(np.float32(GAMMA)) * target_q)
        fetch = ["FullyConnected_9/BiasAdd", "Adam_1", "MeanSquare/Mean"] + \
            [g_critic[k] for k in CRITIC]
        res = sess.run(fetch, {"InputData_2/X": ps, "InputData_3/X": a, "Placeholder_1": y})
        q, loss, gc = res[0], res[2], res[3:]
        a_outs = sess.run(out, {"InputData/X": ps})
        da = sess.run("gradients_2/FullyConnected_7/MatMul_grad/MatMul",
                      {"InputData_2/X": ps, "InputData_3/X": a_outs})
        res = sess.run(["Adam"] + [g_actor[k] for k in ACTOR],
                       {"InputData/X": ps, "Placeholder": da})
        ga = res[1:]
        sess.run(["Assign_%d" % i for i in range(3, 8)])
        sess.run(["Assign_%d" % i for i in range(8, 16)])
        p = "step%d/" % step
        fx.update({p + "s": s, p + "a": a, p + "r": r, p + "t": t, p + "s2": s2,
                   p + "target_q": target_q, p + "y": y, p + "q": q, p + "loss": np.float64(loss),
                   p + "a_outs": a_outs, p + "da": da})
        for k, g in zip(CRITIC, gc):
            fx[p + "grad/" + k] = g.astype(np.float32)
        for k, g in zip(ACTOR, ga):
            fx[p + "grad/" + k] = g.astype(np.float32)
    for k in ACTOR + CRITIC + ACTOR_T + CRITIC_T:
        fx["final/" + k] = sess.vars[k].astype(np.float32)
    for k in ACTOR + CRITIC:
        fx["final/%s/Adam" % k] = sess.vars[k + "/Adam"].astype(np.float32)
        fx["final/%s/Adam_1" % k] = sess.vars[k + "/Adam_1"].astype(np.float32)
    for k in POWERS:
        fx["final/" + k] = np.float64(sess.vars[k])
    if fresh or scaler is not None:
        # the weights the trajectory starts from (model-1410's are in
        # ip_model1410.npz; the MountainCar ones are stored here)
        for k in ACTOR + CRITIC + ACTOR_T + CRITIC_T:
            fx["init/" + k] = state[k].astype(np.float32)
    if scaler is not None:
        fx["scaler/mean"], fx["scaler/scale"] = scaler
    return fx


def ip_batch(rng, b=B):
    """An InvertedPendulum-like batch as the reference's replay returns it."""
    s = rng.normal(0, 0.2, (b, 4))
    s2 = s + rng.normal(0, 0.02, (b, 4))
    a = rng.uniform(-3, 3, (b, 1)).astype(np.float32)
    r = np.ones(b)
    t = rng.random(b) < 0.1
    return s, a, r, t, s2


# MountainCarContinuous-v0 observation box (position, velocity)
MC_LOW, MC_HIGH = np.array([-1.2, -0.07]), np.array([0.6, 0.07])


def mc_scaler():
    """StandardScaler fitted as ddpg.py:184-189 fits it: on 10 000 draws of
    observation_space.sample() (uniform over the box); mean_ and scale_
    (population std) in float64."""
    obs = np.random.default_rng(184).uniform(MC_LOW, MC_HIGH, (10000, 2))
    return obs.mean(axis=0), obs.std(axis=0)


def mc_batch(rng):
    """A MountainCar-like batch: raw (unscaled) float64 states in the box, a
    one-dimensional action in [-1, 1], reward -0.1 a^2 with an occasional
    +100 and done at the goal."""
    s = rng.uniform(MC_LOW, MC_HIGH, (B, 2))
    s2 = np.clip(s + rng.normal(0, [0.01, 0.002], (B, 2)), MC_LOW, MC_HIGH)
    a = rng.uniform(-1, 1, (B, 1)).astype(np.float32)
    t = rng.random(B) < 0.05
    r = -0.1 * a[:, 0].astype(np.float64) ** 2 + 100.0 * t
    return s, a, r, t, s2


def main():
    fx = trajectory(REF, REF, "ip", ip_batch, STEPS)
    np.savez_compressed(os.path.join(HERE, "graph_ip1410.npz"), **fx)
    print("graph_ip1410.npz: %d arrays, loss per step %s" % (
        len(fx), [float(fx["step%d/loss" % i]) for i in range(STEPS)]))
    # Adam bias correction: the same graph and weights with the optimizer state
    # the graph's initializers give (slots 0, beta powers 0.9 / 0.999), so step
    # 1 applies alpha = lr * sqrt(1 - 0.999) / (1 - 0.9) = 0.316 lr
    fx = trajectory(REF, REF, "ip", ip_batch, STEPS, fresh=True)
    np.savez_compressed(os.path.join(HERE, "graph_ip1410_fresh.npz"), **fx)
    print("graph_ip1410_fresh.npz: %d arrays, beta powers after %d steps %s" % (
        len(fx), STEPS, [float(fx["final/" + k]) for k in POWERS]))
    # the MountainCar graph (S=2, actor 48/64, critic 48/128) from its own
    # checkpoint (t ~ 45k Adam steps), states through the fitted scaler
    # the reference's default batch (parameters.py:11, 256): the same graph and
    # checkpoint, 3 steps of 256 rows -- on the GPU this runs through the
    # large-batch GEMM path (DDPG_SMALL=0), pinning the twin GEMMs, their
    # in-launch K split and the slab reductions to the executed graph directly
    fx = trajectory(REF, REF, "ip", lambda rng: ip_batch(rng, 256), STEPS)
    np.savez_compressed(os.path.join(HERE, "graph_ip1410_b256.npz"), **fx)
    print("graph_ip1410_b256.npz: %d arrays, loss per step %s" % (
        len(fx), [float(fx["step%d/loss" % i]) for i in range(STEPS)]))
    fx = trajectory(MC, MC, "mc", mc_batch, STEPS, scaler=mc_scaler())
    np.savez_compressed(os.path.join(HERE, "graph_mc120.npz"), **fx)
    print("graph_mc120.npz: %d arrays, loss per step %s" % (
        len(fx), [float(fx["step%d/loss" % i]) for i in range(STEPS)]))


if __name__ == "__main__":
    main()
