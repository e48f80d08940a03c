"""One rank of tests/test_gpu_dp_shm.py (run as a subprocess, not collected).

  python tests/dp_shm_worker.py <cfg> <dtype> <per-rank batch> <steps> <out.npz>

RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT from the environment (world 1:
the single-process reference, no communicator).  With world > 1 the parent
points DDPG_LIB_PATH at tools/shm/libddpg_shm.so, whose RCCL calls are the
/dev/shm stand-in (tools/rccl_shm.cpp), so N processes share the one GPU.
Saves every parameter / Adam / gradient buffer after the first and the last
step, and the step stats."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    cfg, dtype, b, steps, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    sess, rb, fl, _ = bench.build_learner(cfg, 0, rank, world, 20_000, dtype=dtype, per_gpu_b=b)
    res = {}
    for i in range(steps):
        st = fl.step(stats=True)
        if i in (0, steps - 1):
            res["stats%d" % i] = np.array(st, np.float64)
            for w in range(10):
                res["s%d_w%d" % (i, w)] = sess.get_params(w, split=False)
    res["counts"] = np.array(fl.step_counts(), np.int64)
    from distributed_ddpg_amd import _lib
    res["lib"] = np.array(os.path.basename(_lib.LIB_PATH))
    np.savez(out, **res)
    sess.close()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
