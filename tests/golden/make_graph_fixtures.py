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


def main():
    nodes = tfgraph.read_graph(REF + ".meta")
    state = tfbundle.read_checkpoint(REF)
    sess = tfgraph.Session(nodes, state, dtype=np.float64)
    g_actor = adam_grad_inputs(nodes, "Adam")
    g_critic = adam_grad_inputs(nodes, "Adam_1")
    assert sorted(g_actor) == sorted(ACTOR) and sorted(g_critic) == sorted(CRITIC)
    rng = np.random.default_rng(1410)
    fx = {}
    for k in POWERS:
        fx["init/" + k] = np.float64(state[k])
    for k in ACTOR + CRITIC:
        fx["init/%s/Adam" % k] = state[k + "/Adam"].astype(np.float32)
        fx["init/%s/Adam_1" % k] = state[k + "/Adam_1"].astype(np.float32)
    for step in range(STEPS):
        # an InvertedPendulum-like batch as the reference's replay returns it
        s = rng.normal(0, 0.2, (B, 4))
        s2 = s + rng.normal(0, 0.02, (B, 4))
        a = rng.uniform(-3, 3, (B, 1)).astype(np.float32)
        r = np.ones(B)
        t = rng.random(B) < 0.1
        a2 = sess.run("Mul_1", {"InputData_1/X": s2})
        target_q = sess.run("FullyConnected_13/BiasAdd", {"InputData_4/X": s2,
                                                          "InputData_5/X": a2})
        # GAMMA * target_q[k] multiplies a float32 array in the reference: the
        # Python-float gamma enters as float32 (ddpg.py:97)
        y = np.where(t[:, None], r[:, None], r[:, None] + np.float64(np.float32(GAMMA)) * target_q)
        fetch = ["FullyConnected_9/BiasAdd", "Adam_1", "MeanSquare/Mean"] + \
            [g_critic[k] for k in CRITIC]
        res = sess.run(fetch, {"InputData_2/X": s, "InputData_3/X": a, "Placeholder_1": y})
        q, loss, gc = res[0], res[2], res[3:]
        a_outs = sess.run("Mul", {"InputData/X": s})
        da = sess.run("gradients_2/FullyConnected_7/MatMul_grad/MatMul",
                      {"InputData_2/X": s, "InputData_3/X": a_outs})
        res = sess.run(["Adam"] + [g_actor[k] for k in ACTOR],
                       {"InputData/X": s, "Placeholder": da})
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
    np.savez_compressed(os.path.join(HERE, "graph_ip1410.npz"), **fx)
    print("graph_ip1410.npz: %d arrays, loss per step %s" % (
        len(fx), [float(fx["step%d/loss" % i]) for i in range(STEPS)]))


if __name__ == "__main__":
    main()
