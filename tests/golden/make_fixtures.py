"""Generate the committed golden fixtures under tests/golden/.

Run ONLY in the build container (it reads /root/reference, which does not
exist on the GPU box):   python tests/golden/make_fixtures.py

Outputs (all plain data; nothing from the reference's source travels):
  replay_indices.npz   -- sample indices produced by the reference's own
                          `ReplayBuffer.sample_batch` (replay_buffer.py:33-47),
                          imported from /root/reference, on payload-encoded
                          rows (row i carries i in s[0]) so the drawn deque
                          positions can be read back.  Each case is a script
                          of add/sample ops.
  mc_model120.npz      -- every float tensor of the reference's MountainCar
                          checkpoint results/model_ddpg/model-120 (weights,
                          targets, Adam m/v slots, beta powers).
  ip_model1410.npz     -- weights/targets/beta powers of
                          InvertedPendulum/model_ddpg/model-1410 (Adam slots
                          dropped to keep the fixture small).
  meta_constants.json  -- graph constants decoded from model-1410.meta
                          (Adam lr/betas/eps, tau, action scale, init ranges).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, HERE)
import tfbundle  # noqa: E402

# (name, seed, capacity, ops)  ops: ("add", n) / ("sample", k)
REPLAY_CASES = [
    ("survey_prewrap", 1234, 1000, [("add", 300), ("sample", 8)]),
    ("survey_postwrap", 1234, 100, [("add", 250), ("sample", 8)]),
    ("pool_branch_b64", 1234, 10_000, [("add", 200), ("sample", 64), ("sample", 64)]),
    ("set_branch_b64", 1234, 10_000, [("add", 2000), ("sample", 64)]),
    ("pool_branch_b256", 7, 5000, [("add", 1000), ("sample", 256)]),
    ("set_branch_b256", 7, 5000, [("add", 5000), ("sample", 256), ("sample", 256)]),
    ("tiny_k", 99, 50, [("add", 30), ("sample", 1), ("sample", 5), ("sample", 6)]),
    ("count_lt_batch", 5, 100, [("add", 10), ("sample", 64)]),
    ("interleaved_wrap", 1234, 320,
     [("add", 300), ("sample", 64), ("add", 50), ("sample", 64), ("add", 400), ("sample", 64),
      ("add", 1), ("sample", 256)]),
    ("default_seed_123", 123, 1000, [("add", 999), ("sample", 32)]),
    ("seed_zero", 0, 1000, [("add", 500), ("sample", 16)]),
    ("seed_negative", -77, 1000, [("add", 500), ("sample", 16)]),
    ("seed_multiword", 2 ** 40 + 5, 1000, [("add", 500), ("sample", 16)]),
    ("full_1e6_b4096", 1234, 1_000_000,
     [("add", 1_000_000), ("sample", 4096), ("sample", 4096), ("add", 77), ("sample", 64)]),
]


def make_replay():
    sys.path.insert(0, REF)
    import replay_buffer  # the reference module itself

    a0 = np.zeros(1, np.float32)
    s2 = np.zeros(1)
    arrays = {}
    meta = []
    for name, seed, cap, ops in REPLAY_CASES:
        rb = replay_buffer.ReplayBuffer(cap, seed)
        added = 0
        outs = []
        for op, n in ops:
            if op == "add":
                for i in range(added, added + n):
                    rb.add(np.array([float(i)]), a0, float(i) * 0.5, (i % 7) == 0, s2)
                added += n
            else:
                s, a, r, t, _ = rb.sample_batch(n)
                ins = s[:, 0].astype(np.int64)
                assert np.array_equal(r, ins * 0.5) and np.array_equal(t, ins % 7 == 0)
                outs.append(ins)
        for j, o in enumerate(outs):
            arrays["%s__%d" % (name, j)] = o.astype(np.int64)
        meta.append({"name": name, "seed": seed, "capacity": cap,
                     "ops": [[op, n] for op, n in ops], "n_samples": len(outs)})
    arrays["__cases__"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "replay_indices.npz"), **arrays)
    print("replay_indices.npz: %d cases" % len(meta))


def make_checkpoints():
    mc = tfbundle.read_checkpoint(REF + "/results/model_ddpg/model-120")
    np.savez_compressed(os.path.join(HERE, "mc_model120.npz"), **mc)
    ip = tfbundle.read_checkpoint(REF + "/InvertedPendulum/model_ddpg/model-1410")
    keep = {k: v for k, v in ip.items() if "/Adam" not in k}
    np.savez_compressed(os.path.join(HERE, "ip_model1410.npz"), **keep)
    print("mc_model120.npz: %d tensors; ip_model1410.npz: %d tensors" % (len(mc), len(keep)))


def make_meta_constants():
    version, nodes = tfbundle.read_meta_nodes(REF + "/InvertedPendulum/model_ddpg/model-1410.meta")
    consts = {}
    devices = {}
    ops = {}
    for name, op, dev, attrs in nodes:
        ops[op] = ops.get(op, 0) + 1
        if op == "ApplyAdam":
            devices[name] = dev
        if op != "Const":
            continue
        f = tfbundle.const_float(attrs)
        if f is None:
            continue
        if (name.startswith(("Adam", "beta", "Mul")) or "Square_grad/mul/x" in name
                or "truncated_normal/stddev" in name or "random_uniform/m" in name):
            consts[name] = f
    out = {"tf_version": version, "consts": consts, "apply_adam_devices": devices,
           "op_histogram": ops}
    with open(os.path.join(HERE, "meta_constants.json"), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print("meta_constants.json: tf %s, %d consts" % (version, len(consts)))


if __name__ == "__main__":
    make_meta_constants()
    make_checkpoints()
    make_replay()
