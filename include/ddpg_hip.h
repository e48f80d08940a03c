/*
 * ddpg_hip.h -- C-ABI of the MI355X-native DDPG learner-update hot path.
 *
 * This is the drop-in boundary that replaces the TF 1.3 session calls made by
 * the reference's networks.py / replay_buffer.py.  Every
 * entry point below cites the reference interface it replaces.  No torch or
 * C++ types cross this boundary: plain pointers, sizes and int error codes.
 *
 * Conventions
 *   - Return 0 on success, a negative DDPG_E* code on error; the message is
 *     available from ddpg_last_error(ctx) (or ddpg_global_error() when no ctx
 *     exists yet).  No C++ exception crosses the ABI.
 *   - Host pointers are caller-owned.  Device weights, optimiser state, the
 *     replay ring and workspaces are library-owned.
 *   - One ctx per process per GPU; not thread-safe; all work is ordered on
 *     the ctx's HIP stream.  Calls that return host data synchronise.
 *   - All host arrays are row-major float32 ([rows, cols], cols contiguous),
 *     matching what TF's feed_dict casts the reference's numpy inputs to.
 *   - Parameter vectors are flat float32 in the reference checkpoint order
 *     (SURVEY.md §4.3):  actor  = [W1 (S,H1), b1, W2 (H1,H2), b2, W3 (H2,A)]
 *                        critic = [Ws (S,H1), bs, Wa (A,H1), ba, Wh (2H1,H2),
 *                                  bh, Wo (H2,1), bo (1)]
 */
#ifndef DDPG_HIP_H
#define DDPG_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 2 (behaviour change from 1): the 1:1 methods no longer apply the scaler
 * set by ddpg_set_scaler -- callers pass preprocessed states (see there); only
 * the fused step's replay gathers scale.  Pinned by
 * tests/test_gpu_configs.py::test_mountaincar_scaler_parity (1:1 and fused). */
#define DDPG_ABI_VERSION 2

enum ddpg_status {
  DDPG_OK = 0,
  DDPG_EINVAL = -1,   /* bad argument / shape mismatch (TF InvalidArgumentError) */
  DDPG_EHIP = -2,     /* HIP runtime error */
  DDPG_ENOMEM = -3,   /* allocation failure */
  DDPG_ESTATE = -4,   /* call not valid in the current state */
  DDPG_ECOMM = -5     /* RCCL error */
};

enum ddpg_dtype { DDPG_FP32 = 0, DDPG_BF16 = 1 };

/* which parameter set (ddpg_set_params / ddpg_get_params) */
enum ddpg_which {
  DDPG_ACTOR = 0,       /* ActorNetwork.network_params          networks.py:27 */
  DDPG_ACTOR_TARGET = 1,/* ActorNetwork.target_network_params   networks.py:31 */
  DDPG_CRITIC = 2,      /* CriticNetwork.network_params         networks.py:119 */
  DDPG_CRITIC_TARGET = 3,
  DDPG_ACTOR_ADAM_M = 4,  /* "<var>/Adam"   slots of the actor optimiser */
  DDPG_ACTOR_ADAM_V = 5,  /* "<var>/Adam_1" */
  DDPG_CRITIC_ADAM_M = 6,
  DDPG_CRITIC_ADAM_V = 7,
  /* get only: the gradient the last update applied (after the data-parallel
   * sum), i.e. the `grads` of networks.py:44 / the compute_gradients of
   * networks.py:137, in the same flat order */
  DDPG_ACTOR_GRAD = 8,
  DDPG_CRITIC_GRAD = 9
};

/* ddpg_replay_create_ex flags */
#define DDPG_REPLAY_F64 1  /* keep s, s2, r as float64 (the reference's deque values) */

/* soft-update mask (ddpg_soft_update) */
#define DDPG_SOFT_ACTOR 1
#define DDPG_SOFT_CRITIC 2

typedef struct ddpg_cfg {
  int state_dim;      /* S */
  int action_dim;     /* A */
  int h1, h2;         /* actor hidden widths (reference: 128 / 200, networks.py:54-55) */
  int batch_max;      /* max rows per call (per rank) */
  float actor_lr;     /* parameters.py:15  (1e-4) */
  float critic_lr;    /* parameters.py:14  (1e-3) */
  float tau;          /* parameters.py:17  (1e-3) */
  float gamma;        /* parameters.py:13  (0.99) */
  float action_scale; /* |action_space.high| ddpg.py:196-197 */
  float beta1, beta2, epsilon; /* TF AdamOptimizer defaults 0.9/0.999/1e-8 */
  int dtype;          /* ddpg_dtype: GEMM operand precision (fp32 master state always) */
  int device;         /* HIP device ordinal */
  int rank, world;    /* data-parallel position; world==1 -> no collectives */
  int critic_h1, critic_h2; /* critic widths (networks.py:151-156); 0 = same as actor.
                             * The reference's MountainCar checkpoint uses 48/64 vs 48/128. */
} ddpg_cfg;

typedef struct ddpg_ctx ddpg_ctx;
typedef struct ddpg_replay ddpg_replay;
typedef struct ddpg_sampler ddpg_sampler;

typedef struct ddpg_stats {
  float q_max;        /* np.amax(predicted_q_value)   ddpg.py:102 */
  float loss;         /* v_loss                        ddpg.py:103 */
} ddpg_stats;

/* ------------------------------------------------------------- lifecycle */
int ddpg_abi_version(void);
const char* ddpg_global_error(void);
/* ActorNetwork.__init__ + CriticNetwork.__init__ + tf.Session (networks.py:17,109; ddpg.py:237) */
int ddpg_create(const ddpg_cfg* cfg, ddpg_ctx** out);
void ddpg_destroy(ddpg_ctx* ctx);
const char* ddpg_last_error(ddpg_ctx* ctx);
int ddpg_sync(ddpg_ctx* ctx);
/* Use an external HIP stream (e.g. torch's current stream); NULL = own stream. */
int ddpg_set_stream(ddpg_ctx* ctx, void* hip_stream);

/* ------------------------------------------------------------- parameters */
/* number of floats of a parameter set in checkpoint order */
int ddpg_param_count(ddpg_ctx* ctx, int which, size_t* n);
/* restore_params / saver.restore (networks.py:93-96, 201-204; ddpg.py:217) */
int ddpg_set_params(ddpg_ctx* ctx, int which, const float* host, size_t n);
int ddpg_get_params(ddpg_ctx* ctx, int which, float* host, size_t n);
/* beta1_power / beta2_power (net: 0 actor, 1 critic) and the Adam step count */
int ddpg_set_adam_powers(ddpg_ctx* ctx, int net, float beta1_power, float beta2_power);
int ddpg_get_adam_powers(ddpg_ctx* ctx, int net, float* beta1_power, float* beta2_power);

/* ------------------------------------------------------------- 1:1 methods */
/* ActorNetwork.predict / predict_target          networks.py:77-85 */
int ddpg_actor_forward(ddpg_ctx* ctx, int target, const float* s, int B, float* a_out);
/* CriticNetwork.predict / predict_target         networks.py:177-187 */
int ddpg_critic_forward(ddpg_ctx* ctx, int target, const float* s, const float* a, int B,
                        float* q_out);
/* CriticNetwork.train -> [out (pre-update), optimize, loss]   networks.py:170-175 */
int ddpg_critic_train(ddpg_ctx* ctx, const float* s, const float* a, const float* y, int B,
                      float* q_pre, float* loss);
/* CriticNetwork.action_gradients (grad_ys = 1)   networks.py:143,189-193 */
int ddpg_critic_action_grad(ddpg_ctx* ctx, const float* s, const float* a, int B, float* da);
/* ActorNetwork.train(inputs, a_gradient)          networks.py:39-47,71-75 */
int ddpg_actor_train(ddpg_ctx* ctx, const float* s, const float* a_gradient, int B);
/* update_target_network (mask: DDPG_SOFT_*)        networks.py:34-37,87-88,126-128,195-196 */
int ddpg_soft_update(ddpg_ctx* ctx, int mask);
/* per-feature affine input scaler (sklearn StandardScaler.transform, ddpg.py:184-189,
 * networks.py:65-69,164-168): (x - mean) / scale in float64, then one rounding to
 * fp32.  Applied ONLY where the library reads raw replay rows (the fused
 * learner step's gathers).  The 1:1 methods above take states that the caller
 * already preprocessed (the shims' preprocess_input, float64 on the host), as
 * the reference's feed_dict received them.  NULL clears. */
int ddpg_set_scaler(ddpg_ctx* ctx, const double* mean, const double* scale, int S);

/* ------------------------------------------------------------- replay */
/* Host restatement of CPython random.seed(int) + random.sample (MT19937),
 * the sampler behind ReplayBuffer.sample_batch (replay_buffer.py:19,33-39). */
int ddpg_sampler_create(int64_t seed, ddpg_sampler** out);
void ddpg_sampler_destroy(ddpg_sampler* s);
/* k indices drawn uniformly without replacement from range(n), exactly as
 * random.sample(range(n), k) would return them. */
int ddpg_sampler_sample(ddpg_sampler* s, int64_t n, int k, int64_t* out);
/* raw MT19937 state words (624) + position, for tests */
int ddpg_sampler_getrandbits32(ddpg_sampler* s, uint32_t* out, int n);

/* Device ring buffer of transitions (ReplayBuffer replay_buffer.py:10-51).
 * Rows: s[S], a[A], r, t, s2[S]; a fp32, t as 0/1; s, s2, r fp32, or float64
 * with DDPG_REPLAY_F64 (what the reference's deque holds when the env emits
 * float64 states: sample_batch then returns them exactly and the scaler sees
 * the unrounded state).  The learner rounds them to fp32 once, as TF's
 * feed_dict does. */
int ddpg_replay_create(int device, int state_dim, int action_dim, int64_t capacity,
                       int64_t seed, ddpg_replay** out);
int ddpg_replay_create_ex(int device, int state_dim, int action_dim, int64_t capacity,
                          int64_t seed, int flags, ddpg_replay** out);
int ddpg_replay_is_f64(ddpg_replay* rb);
void ddpg_replay_destroy(ddpg_replay* rb);
const char* ddpg_replay_last_error(ddpg_replay* rb);
/* ReplayBuffer.add (replay_buffer.py:21-28), n rows at once (host arrays) */
int ddpg_replay_add(ddpg_replay* rb, const float* s, const float* a, const float* r,
                    const uint8_t* t, const float* s2, int n);
/* the same with float64 s, r, s2 (rounded to fp32 when the ring is fp32) */
int ddpg_replay_add_f64(ddpg_replay* rb, const double* s, const float* a, const double* r,
                        const uint8_t* t, const double* s2, int n);
/* ReplayBuffer.size (replay_buffer.py:30-31) */
int64_t ddpg_replay_size(ddpg_replay* rb);
int64_t ddpg_replay_total_added(ddpg_replay* rb);
/* ReplayBuffer.clear (replay_buffer.py:49-51; the reference's is broken) */
int ddpg_replay_clear(ddpg_replay* rb);
/* ReplayBuffer.sample_batch (replay_buffer.py:33-47): draws min(B, size)
 * deque positions with the buffer's sampler and gathers the rows to host.
 * Returns the number of rows (>=0) or an error. idx_out (optional) receives
 * the deque positions. */
int ddpg_replay_sample_batch(ddpg_replay* rb, int B, float* s, float* a, float* r,
                             uint8_t* t, float* s2, int64_t* idx_out);
/* the same with float64 s, r, s2 outputs (exact for a DDPG_REPLAY_F64 ring) */
int ddpg_replay_sample_batch_f64(ddpg_replay* rb, int B, double* s, float* a, double* r,
                                 uint8_t* t, double* s2, int64_t* idx_out);

/* ------------------------------------------------------------- fused path */
/* One whole learner step, ddpg.py:86-113, on device: sample (host MT19937)
 * -> gather (K8) -> target actor/critic fwd + TD target (K1,K2,K9) ->
 * critic train (K2,K3,K6) -> actor fwd + dQ/da (K1,K4) -> actor train
 * (K5,K6) -> both soft updates (K7).  B is the GLOBAL batch; with world>1
 * this rank processes rows [rank*B/world, (rank+1)*B/world) and gradients
 * are summed over ranks with RCCL; with a communicator the stats are the
 * global-batch ones (max over ranks of max(Q), sum of the loss shares).
 * stats may be NULL (no host sync).  Argument errors (replay dims, B outside
 * [1, batch_max] per rank or not divisible by world, fewer than B rows) return
 * a negative status BEFORE anything moves: the sampler, parameters and Adam
 * state are as they were. */
int ddpg_learner_step(ddpg_ctx* ctx, ddpg_replay* rb, int B, ddpg_stats* stats);
/* Same, with an explicit host index list (deque positions, length B). */
int ddpg_learner_step_indices(ddpg_ctx* ctx, ddpg_replay* rb, const int64_t* idx, int B,
                              ddpg_stats* stats);
/* Accumulated per-step stats on device since last reset:
 * sum of q_max, sum of loss, steps (ddpg.py:102-103, 121-122). */
int ddpg_read_stats(ddpg_ctx* ctx, double* q_max_sum, double* loss_sum, int64_t* steps,
                    int reset);

/* ------------------------------------------------------------- multi-GPU */
/* RCCL unique id (128 bytes) on rank 0; broadcast it out of band. */
int ddpg_comm_unique_id(char* out128);
/* Replaces tf.train.ClusterSpec/Server + replica_device_setter (ddpg.py:168-174).
 * world/rank must equal the cfg's.  world == 1 creates a 1-rank communicator:
 * the step then runs its exchanges through the same RCCL call sites (identity
 * sums) on the large-batch path -- a test of those call sites on one GPU;
 * without a communicator a world == 1 ctx issues no collectives.
 * The exchanges run on a library-owned comm stream: the dWh (critic) and dW2
 * (actor) all-reduces start as soon as those gradients are reduced, under the
 * remaining backward GEMMs; each network's Adam waits for its exchange.  The
 * step's hipGraph captures the RCCL calls with the kernels (env
 * DDPG_GRAPH_COMM=0, or a failed capture, keeps such steps eager). */
int ddpg_comm_init(ddpg_ctx* ctx, const char* id128, int world, int rank);
/* Measurement hook (bench.py --per-rank-of): a 1-rank communicator standing in
 * for the cfg.world-rank one, so that ONE GPU runs exactly rank cfg.rank's
 * share of a cfg.world-rank step -- its slice of the global draw, every RCCL
 * call site (as identities), the same issue path -- for timing.  Gradients are
 * then this rank's partial sums, not the global ones. */
int ddpg_comm_init_proxy(ddpg_ctx* ctx);

/* How this ctx's learner steps ran so far: replayed from the step's hipGraph
 * or launched eagerly, and whether a capture with RCCL calls failed (the ctx
 * then runs its data-parallel steps eagerly).  Any pointer may be NULL. */
int ddpg_step_counts(ddpg_ctx* ctx, int64_t* graphed, int64_t* eager, int* capture_failed);

/* ------------------------------------------------------------- profiling */
/* Enable per-kernel HIP-event timing on the ctx stream (0 disables). */
int ddpg_profile_enable(ddpg_ctx* ctx, int enable);
/* Per-kernel-class totals since enable: fills up to n entries of names (each
 * <=63 chars), total ms, launches and algorithmic flop / bytes. Returns count. */
int ddpg_profile_read(ddpg_ctx* ctx, int n, char (*names)[64], double* ms, int64_t* launches,
                      double* flops, double* bytes);

/* ------------------------------------------------------------- checkpoints */
/* CRC-32C (Castagnoli) of n bytes continuing from crc (0 to start): the checksum
 * of TF V2 checkpoint blocks and tensors, for the tf.train.Saver work-alike
 * (distributed_ddpg_amd/checkpoint.py; replaces TF's Saver.save/restore,
 * ddpg.py:155-159, 211-222).  Host only, thread-safe. */
uint32_t ddpg_crc32c(uint32_t crc, const void* data, size_t n);

#ifdef __cplusplus
}
#endif
#endif /* DDPG_HIP_H */
