"""Episode driver with the reference's CLI contract (ddpg.py:16-19, 162-270):

    python -m distributed_ddpg_amd.ddpg --job_name=ps     --task_index=0
    python -m distributed_ddpg_amd.ddpg --job_name=worker --task_index=0

`ps` hosts the rendezvous store at Parameters.parameter_servers[0] and blocks
(the reference's server.join(), ddpg.py:171-172).  Each `worker` i becomes
rank i of a synchronous data-parallel group of len(Parameters.workers) ranks:
one GPU per worker (LOCAL device = task_index unless --device), gradients
summed with RCCL inside the fused learner step.  The reference's workers
apply asynchronous Hogwild updates on the PS; that semantics is deliberately
replaced.

Per environment step the worker does what ddpg.py:66-116 does: act with
actor.predict(s) + 1/(1+global_step), store the transition, and -- once the
buffer holds more than batch_size rows -- one learner update (the fused
device path, ddpg_learner_step).  gym/MuJoCo are used when importable; this
image has neither, so --env synthetic (default when gym is missing) provides
an InvertedPendulum-shaped stand-in environment.
"""
import argparse
import os
import sys
import time

import numpy as np


class SyntheticEnv:
    """Stand-in continuous-control task shaped like InvertedPendulum-v1
    (obs 4, action 1 in [-3, 3], reward 1 per step, termination when the
    state leaves a box, 1000-step limit)."""

    class _Box:
        def __init__(self, low, high, shape):
            self.low = np.full(shape, low, np.float64)
            self.high = np.full(shape, high, np.float64)
            self.shape = shape

        def sample(self, rng=np.random):
            return rng.uniform(self.low, self.high)

    def __init__(self, obs_dim=4, act_dim=1, act_high=3.0, seed=0, max_steps=1000):
        self.observation_space = self._Box(-1.0, 1.0, (obs_dim,))
        self.action_space = self._Box(-act_high, act_high, (act_dim,))
        self.rng = np.random.default_rng(seed)
        A = self.rng.standard_normal((obs_dim, obs_dim)) * 0.05
        self.A = np.eye(obs_dim) + A
        self.Bm = self.rng.standard_normal((obs_dim, act_dim)) * 0.02
        self.max_steps = max_steps

    def reset(self):
        self.t = 0
        self.s = self.rng.uniform(-0.01, 0.01, self.observation_space.shape)
        return self.s.copy()

    def step(self, a):
        a = np.clip(np.asarray(a, np.float64).reshape(-1), self.action_space.low,
                    self.action_space.high)
        self.s = self.A @ self.s + self.Bm @ a + self.rng.standard_normal(self.s.shape) * 1e-3
        self.t += 1
        done = bool(np.any(np.abs(self.s) > 1.0) or self.t >= self.max_steps)
        return self.s.copy(), 1.0, done, {}


def make_env(name, seed):
    if name == "synthetic":
        return SyntheticEnv(seed=seed)
    try:
        import gym
    except ImportError:
        print("gym not installed: using the synthetic InvertedPendulum-shaped environment",
              file=sys.stderr)
        return SyntheticEnv(seed=seed)
    return gym.make(name)


def _host_port(addr):
    host, port = addr.rsplit(":", 1)
    return ("127.0.0.1" if host == "localhost" else host), int(port)


def run_ps(opt):
    """ddpg.py:171-172 -- host the rendezvous store and block."""
    from torch.distributed import TCPStore
    host, port = _host_port(opt.parameter_servers[0])
    store = TCPStore(host, port, world_size=len(opt.workers) + 1, is_master=True,
                     wait_for_workers=False)
    print("ps: rendezvous store at %s:%d for %d workers" % (host, port, len(opt.workers)))
    store.set("ps_ready", "1")
    while True:  # server.join()
        time.sleep(3600)


def rendezvous(opt, rank):
    """Join the ps-hosted store as worker `rank` of len(opt.workers) and form
    the gloo group the RCCL unique id travels over (the reference's
    ClusterSpec + Server, ddpg.py:168-174).  Returns the world size."""
    import torch.distributed as dist
    from torch.distributed import TCPStore
    world = len(opt.workers)
    if world > 1:
        host, port = _host_port(opt.parameter_servers[0])
        store = TCPStore(host, port, world_size=world + 1, is_master=False)
        dist.init_process_group("gloo", store=store, rank=rank, world_size=world)
    return world


def rendezvous_check(opt, rank):
    """--rendezvous_only: the launch path up to the unique-id exchange without
    a GPU.  Rank 0 broadcasts a 128-byte id (random bytes standing in for
    ncclGetUniqueId, which needs the HIP runtime) over the gloo group exactly
    as learner.init_comm does; every rank then reports the id it received."""
    import torch.distributed as dist
    world = rendezvous(opt, rank)
    obj = [os.urandom(128) if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(obj, src=0)
        ids = [None] * world
        dist.all_gather_object(ids, obj[0])
        assert all(i == obj[0] for i in ids), "unique id differs across ranks"
        dist.destroy_process_group()
    print("rendezvous ok rank %d of %d id %s" % (rank, world, obj[0][:8].hex()), flush=True)


def run_worker(opt, task_index, env_name, episodes, device):
    import torch
    import torch.distributed as dist

    from . import checkpoint, networks as nets, summary
    from .learner import FusedLearner, init_comm
    from .replay_buffer import ReplayBuffer

    rank = task_index
    np.random.seed(opt.seed)
    torch.cuda.set_device(device)
    world = rendezvous(opt, rank)

    env = make_env(env_name, opt.seed + rank)
    scaler = None
    if env_name == "MountainCarContinuous-v0":  # ddpg.py:184-189
        from sklearn.preprocessing import StandardScaler
        ex = np.array([env.observation_space.sample() for _ in range(10000)])
        scaler = StandardScaler().fit(ex)
    replay = ReplayBuffer(opt.rm_size, opt.seed, device=device)
    S = env.observation_space.shape[0]
    A = env.action_space.shape[0]
    if abs(env.action_space.low[0]) != abs(env.action_space.high[0]):
        sys.exit("Error: Action space in current environment is asymmetric! ")
    scale = abs(env.action_space.high[0])
    H1, H2 = opt.hidden
    actor = nets.ActorNetwork(S, A, scale, opt.actor_lr, opt.tau, scaler, h1=H1, h2=H2)
    critic = nets.CriticNetwork(S, A, opt.critic_lr, opt.tau, actor.get_num_trainable_vars(),
                                scaler, h1=H1, h2=H2)
    sess = nets.Session(device=device, batch_max=max(opt.batch_size // world, 1), rank=rank,
                        world=world)
    sess.run(nets.global_variables_initializer(seed=opt.seed))
    actor.set_session(sess)
    critic.set_session(sess)
    saver = checkpoint.Saver(max_to_keep=5)                     # ddpg.py:211
    global_step = 0
    latest = checkpoint.latest_checkpoint(opt.save_dir) if opt.continue_training else None
    if latest:                                                   # ddpg.py:213-222
        global_step = int(float(saver.restore(sess, latest)["global_step"]))
        print("Model Restored from %s" % latest, flush=True)
    else:
        actor.update_target_network()   # ddpg.py:227-229
        critic.update_target_network()
    init_comm(sess, rank, world)
    learner = FusedLearner(sess, replay, opt.batch_size)
    is_chief = rank == 0
    writer = summary.FileWriter(opt.summary_dir) if is_chief else None   # ddpg.py:241

    # Flat loop over environment steps: every rank performs exactly one
    # learner update per env step once warm, so the collectives inside the
    # fused step pair up across ranks; the stop decision is agreed by all.
    stats = []
    episode, t = 0, 0
    state = env.reset()
    ep_reward, ep_q, ep_loss = 0.0, 0.0, 0.0
    solved = False
    while True:
        # exploration offset 1/(1 + global_step): global_step is the episode
        # counter restored from the checkpoint (ddpg.py:69, 250)
        a = actor.predict(np.reshape(state, (1, S))) + (1.0 / (1.0 + global_step))
        state2, r, done, _ = env.step(a[0])
        replay.add(np.reshape(state, (S,)), np.reshape(a, (A,)), r, done,
                   np.reshape(state2, (S,)))
        state = state2
        ep_reward += r
        if replay.size() > opt.batch_size:
            q_max, loss = learner.step(stats=True)
            ep_q += q_max
            ep_loss += loss
        t += 1
        if done:
            stats.append(ep_reward)
            if is_chief:  # ddpg.py:118-127
                # the reference divides by its 0-based step index at `done`
                # (steps - 1); a one-step episode would divide by zero there,
                # so that case divides by 1
                div = float(max(t - 1, 1))
                writer.add_episode(global_step, ep_reward, ep_q / div, ep_loss / div)
                writer.flush()
                print("Episode: %d - Iterations: %d - Reward: %f - Qmax: %f - Loss: %f" % (
                    global_step, t - 1, ep_reward, ep_q / div, ep_loss / div), flush=True)
            if np.mean(stats[-100:]) > 950 and len(stats) >= 101:  # ddpg.py:255-260
                print(np.mean(stats[-100:]))
                print("Solved.")
                solved = True
                if is_chief:
                    saver.save(sess, opt.save_dir + "/model", global_step=global_step)
            elif is_chief and episode % opt.valid_freq == opt.valid_freq - 1:  # ddpg.py:262-264
                saver.save(sess, opt.save_dir + "/model", global_step=global_step)
            global_step += 1  # ddpg.py:267 step_op
            episode += 1
            t = 0
            ep_reward, ep_q, ep_loss = 0.0, 0.0, 0.0
            state = env.reset()
        stop = solved or episode >= episodes
        if world > 1:
            flag = torch.tensor([1 if stop else 0])
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
            stop = bool(flag.item())
        if stop:
            break
    if writer:
        writer.close()
    sess.close()
    if world > 1:
        dist.destroy_process_group()
    print("Done")


def main(argv=None):
    from .parameters import Parameters
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--job_name", default="", help="Either 'ps' or 'worker'")
    ap.add_argument("--task_index", type=int, default=0, help="Index of task within the job")
    ap.add_argument("--env", default=None, help="gym id or 'synthetic'")
    ap.add_argument("--episodes", type=int, default=None)
    ap.add_argument("--device", type=int, default=None)
    ap.add_argument("--workers", default=None,
                    help="comma-separated worker addresses (default Parameters.workers)")
    ap.add_argument("--ps", default=None,
                    help="parameter-server (rendezvous) address (default Parameters.parameter_servers[0])")
    ap.add_argument("--rendezvous_only", action="store_true",
                    help="worker: join the group, exchange the unique id, exit (no GPU)")
    args = ap.parse_args(argv)
    opt = Parameters()
    if args.workers:
        opt.workers = args.workers.split(",")
        opt.num_workers = len(opt.workers)
    if args.ps:
        opt.parameter_servers = [args.ps]
    if args.job_name == "ps":
        run_ps(opt)
    elif args.job_name == "worker" and args.rendezvous_only:
        rendezvous_check(opt, args.task_index)
    elif args.job_name == "worker":
        env = args.env or opt.env_name
        run_worker(opt, args.task_index, env, args.episodes or opt.max_episodes,
                   args.task_index if args.device is None else args.device)
    else:
        sys.exit("--job_name must be 'ps' or 'worker'")


if __name__ == "__main__":
    main()
