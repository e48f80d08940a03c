"""Hyper-parameters with the reference's field names and defaults
(parameters.py:5-34).  The hot-path fields are seed, batch_size, rm_size,
gamma, critic_lr, actor_lr and tau; the rest configure the episode driver."""


class Parameters:
    def __init__(self):
        self.seed = 1234

        self.max_exploration_episodes = 500
        self.batch_size = 256          # batch size during training
        self.rm_size = 1000000         # memory replay maximum size
        self.gamma = 0.99              # discount factor
        self.critic_lr = 0.001         # learning rate for critic
        self.actor_lr = 0.0001         # learning rate for actor

        self.tau = 0.001               # moving average for target network

        self.max_episodes = 50000

        self.valid_freq = 100
        self.train_steps = 5

        self.train = True
        self.continue_training = False

        self.env_name = 'InvertedPendulum-v1'   # 'MountainCarContinuous-v0'

        self.summary_dir = './InvertedPendulum/tboard_ddpg'
        self.save_dir = './InvertedPendulum/model_ddpg'

        self.parameter_servers = ["localhost:2222"]
        self.workers = ["localhost:2223"]
        self.num_workers = len(self.workers)

        # MI355X build additions (not in the reference)
        self.hidden = (128, 200)        # networks.py:54-55,151-156
        self.device = 0
