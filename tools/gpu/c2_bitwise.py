"""GPU box: run the small-batch path for a few steps and dump every network's
parameters, to compare two builds bitwise (DDPG_LIB_PATH=tools/abr6/lib<X>.so).
  python tools/gpu/c2_bitwise.py <tag>          -> gpurun_out/c2bw_<tag>.npz
  python tools/gpu/c2_bitwise.py --cmp <a> <b>  -> bitwise comparison"""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())

if sys.argv[1] == "--cmp":
    a = np.load("gpurun_out/c2bw_%s.npz" % sys.argv[2])
    b = np.load("gpurun_out/c2bw_%s.npz" % sys.argv[3])
    bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
    for k in bad:
        d = np.abs(a[k].astype(np.float64) - b[k]).max()
        print("DIFF", k, "max abs", d, "max |x|", np.abs(a[k]).max())
    print("bitwise equal" if not bad else "%d of %d arrays differ" % (len(bad), len(a.files)))
    sys.exit(1 if bad else 0)

import bench  # noqa: E402

out = {}
for B in (64, 50, 256):
    sess, rb, fl, _ = bench.build_learner("c2", 0, 0, 1, 20_000, per_gpu_b=B)
    st = [fl.step(stats=True) for _ in range(6)]
    out["stats_%d" % B] = np.array(st, np.float64)
    for w in range(4):
        out["p%d_%d" % (w, B)] = sess.get_params(w, split=False)
    sess.close()
np.savez("gpurun_out/c2bw_%s.npz" % sys.argv[1], **out)
print("saved", sys.argv[1], len(out))
