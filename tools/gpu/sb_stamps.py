"""GPU box diagnostic: per-level s_memtime stamps of the small-batch (C2) step
(env DDPG_SB_STAMPS=1 makes ddpg_sync print them for the last step)."""
import os, sys
os.environ["DDPG_SB_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench
sess, rb, fl, _ = bench.build_learner("c2", 0, 0, 1, 100000)
for i in range(30):
    fl.step()
    if i >= 25:
        sess.sync()
