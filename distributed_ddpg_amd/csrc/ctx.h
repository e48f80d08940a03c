// Internal interface of libddpg_hip.so shared by its translation units (not
// part of the C-ABI; include/ddpg_hip.h is the boundary).
//   gemm.hip    GEMM / thin-K / skinny-wgrad planning and launches (the
//               plan: tiles, split-K, the small-M in-launch K split, XCD order)
//   step.hip    the learner step's building blocks, the fused step (graphs,
//               small-batch path), the 1:1 reference methods
//   dp.hip      the data-parallel exchange (RCCL on the comm stream)
//   replay.hip  the device replay ring and the MT19937 sampler ABI
//   abi.hip     lifecycle, parameter I/O, profiling, errors
// See DESIGN.md for the data layout and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/ddpg_hip.h"
#include "common.h"
#include "sampler.h"
#include "types.h"

using namespace ddpg;

// ====================================================================== errors
extern thread_local std::string g_err;  // abi.hip

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      throw DdpgError(DDPG_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e));    \
  } while (0)

struct DdpgError {
  int code;
  std::string msg;
  DdpgError(int c, std::string m) : code(c), msg(std::move(m)) {}
};

static DdpgError einval(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  return DdpgError(DDPG_EINVAL, buf);
}

static inline int rup(int x, int m) { return (x + m - 1) / m * m; }

// ====================================================================== layout
// Flat parameter layout: actor tensors then critic tensors, each tensor
// starting on a 64-float (256 B) boundary.  theta / target / m / v / grad all
// share it, so Adam and the soft update are single coalesced passes.
struct Tensor {
  int rows, cols;  // cols == 1 and rows == n for vectors
  size_t off;      // float offset in the flat buffer
  size_t count() const { return (size_t)rows * cols; }
};

enum { AW1, AB1, AW2, AB2, AW3, NA };
enum { CWS, CBS, CWA, CBA, CWH, CBH, CWO, CBO, NC };

struct Layout {
  Tensor a[NA], c[NC];
  size_t actor_begin, actor_end, critic_begin, critic_end, total;
  void build(int S, int A, int H1, int H2, int CH1, int CH2) {
    size_t off = 0;
    auto place = [&](Tensor& t, int r, int c) {
      t.rows = r;
      t.cols = c;
      t.off = off;
      off += ((size_t)r * c + 63) / 64 * 64;
    };
    actor_begin = 0;
    place(a[AW1], S, H1);
    place(a[AB1], H1, 1);
    place(a[AW2], H1, H2);
    place(a[AB2], H2, 1);
    place(a[AW3], H2, A);
    actor_end = critic_begin = off;
    place(c[CWS], S, CH1);
    place(c[CBS], CH1, 1);
    place(c[CWA], A, CH1);
    place(c[CBA], CH1, 1);
    place(c[CWH], 2 * CH1, CH2);
    place(c[CBH], CH2, 1);
    place(c[CWO], CH2, 1);
    place(c[CBO], 1, 1);
    critic_end = total = off;
  }
};

// ====================================================================== profiler
struct ProfRec {
  std::string name;
  hipEvent_t e0, e1;
  double flops, bytes;
};
struct ProfAgg {
  double ms = 0, flops = 0, bytes = 0;
  int64_t launches = 0;
};

// ====================================================================== replay
struct ddpg_replay {
  int device = 0, S = 0, A = 0;
  // f64: s, s2 and r are kept as float64, the values the reference's deque
  // holds (replay_buffer.py:22-26), so sample_batch returns them exactly and
  // the scaler sees the unrounded state; a / t are fp32 / 0-1 either way.
  bool f64 = false;
  int64_t cap = 0, count = 0, total = 0;
  float *ra = nullptr, *rt = nullptr;
  float *rs = nullptr, *rr = nullptr, *rs2 = nullptr;      // fp32 ring
  double *rsd = nullptr, *rrd = nullptr, *rs2d = nullptr;  // float64 ring
  Sampler sampler;
  hipStream_t stream = nullptr;
  std::string err;
  // host staging for single-row adds (s, s2, r in the ring's precision)
  std::vector<unsigned char> st_s, st_s2, st_r;
  std::vector<float> st_a, st_t;
  int64_t st_first = 0;  // insertion index of first staged row
  int st_n = 0;
  std::vector<int64_t> tmp_idx;
  std::vector<int> tmp_slot;
  int* d_slots = nullptr;
  int d_slots_cap = 0;
  unsigned char* d_tmp = nullptr;
  size_t d_tmp_cap = 0;
  // recorded by learner contexts after their gather; ring writes wait on it so
  // a queued gather never reads rows that a later add overwrote
  hipEvent_t last_read = nullptr;
  // small flushes (a worker's few rows per step) travel in a kernel's
  // arguments, asynchronously; learner steps wait on `written` before their
  // gather.  DDPG_RING_ARGS=0: copies from the host staging plus a stream wait.
  hipEvent_t written = nullptr;
  bool written_rec = false;  // `written` recorded at least once
  uint64_t written_by = 0;  // ddpg_ctx::uid whose stream `written` was last recorded on
  bool args_flush = true;
  explicit ddpg_replay(int64_t seed) : sampler(seed) {}
  size_t es() const { return f64 ? 8 : 4; }  // bytes per s / s2 / r element
  unsigned char* ps() const { return f64 ? (unsigned char*)rsd : (unsigned char*)rs; }
  unsigned char* ps2() const { return f64 ? (unsigned char*)rs2d : (unsigned char*)rs2; }
  unsigned char* pr() const { return f64 ? (unsigned char*)rrd : (unsigned char*)rr; }
};

// on / by: the stream and context uid of the learner step about to read the
// ring (the small, kernel-argument form then runs in that stream's order), or
// null / 0
// ddpg_sync (step.hip): everything queued on c->stream has finished
struct ddpg_ctx;
void sync_stream(ddpg_ctx* c);
void replay_flush(ddpg_replay* rb, hipStream_t on = nullptr, uint64_t by = 0);

// ====================================================================== context
// a GEMM queued under gemm_defer (gemm_flush)
struct DeferredGemm {
  GemmHArgs a;
  dim3 grid;
  double flops, bytes;
  char key[112];
};

struct ddpg_ctx {
  ddpg_cfg cfg{};
  uint64_t uid = 0;  // unique per context for the process lifetime (never reused)
  Layout L;
  int S, A, AH1, AH2, CH1, CH2, Bmax;
  int ldS, ldA, ldAH1, ldAH2, ldCH2, ldC;
  hipStream_t stream = nullptr;
  bool own_stream = true;
  // launch target of the building blocks: == stream except inside the fused
  // step, which forks independent branches onto aux[0..1] (fork/join events;
  // captured into the step's hipGraph like any other dependency)
  hipStream_t cur = nullptr;
  hipStream_t aux[2] = {nullptr, nullptr};
  hipEvent_t fj[8] = {};
  std::string err;

  // parameters (fp32 master) -- one allocation: theta|target|m|v|grad
  float* dparams = nullptr;
  float *theta = nullptr, *target = nullptr, *adam_m = nullptr, *adam_v = nullptr,
        *grad = nullptr;
  float* dpw = nullptr;          // [actor b1p, b2p, critic b1p, b2p]
  unsigned* dcounter = nullptr;  // [2]
  float* dstats = nullptr;       // [q_max, loss]
  float* dstats_all = nullptr;   // [world][2] all-gathered stats (world > 1)
  __bf16* xbuf = nullptr;        // bf16 configuration: the exchange's bf16 payload (L.total)
  float* xrs = nullptr;          // bf16 configuration: this rank's fp32 reduce-scatter slices
  double* dacc = nullptr;        // [qmax_sum, loss_sum, steps]
  double *dmean = nullptr, *dscale = nullptr;
  bool has_scaler = false;

  // activations / workspaces
  float* dact = nullptr;
  float *s, *s2, *a, *r, *t, *y, *q, *dq;
  float *th1, *tcat, *ta2, *cat, *h, *dhp, *dcat;
  float *h1, *h2, *o, *mu, *cat2, *dhp2, *da, *dz3, *dz2, *dz1, *dain;
  float *ppart, *qpart, *colpart, *headpart;  // partial-sum scratch
  float2* lpart = nullptr;                    // loss-kernel block partials
  float *ppart_t, *qpart_t;                   // target-path copies (concurrent branch)
  float *slab_W1, *slab_W2, *slab_W3, *slab_Ws, *slab_Wa, *slab_Wh;
  // per-row-tile partials of the narrow weight gradients fused into the dX
  // epilogues (GemmEpi.nw_*; null: not fused)
  float *nw_W1 = nullptr, *nw_Ws = nullptr, *nw_Wa = nullptr;
  // per-row-tile partials of dW3 fused into thin_k's dz2 launch (TkPart.dw)
  float* tk_dW3 = nullptr;
  // bf16 twins (gemm_h.h operands): hnp planes (0 off, 1 bf16 config, 3 the
  // exact h/m/l split of fp32).  Parameters: theta's twin at wtw, the
  // target's at wtw + hnp * PT (planes PT apart), current while wtw_ok.
  // Activations: atw mirrors dact (planes act_n apart); only the buffers in
  // `twinned` are written (by their producers) and read.
  int hnp = 0;
  __bf16* wtw = nullptr;
  bool wtw_ok = false;
  __bf16* atw = nullptr;
  size_t act_n = 0;
  std::vector<std::pair<const float*, size_t>> twinned;
  int split_cap_W1, split_cap_W2, split_cap_W3, split_cap_Ws, split_cap_Wa, split_cap_Wh;
  // the step's replay slots as the gather / phase kernels read them: the
  // pinned host buffer the sampler filled (device-readable; no upload), or
  // d_slots after a hipMemcpyAsync with DDPG_SLOTS_H2D=1
  const int* slots_src = nullptr;
  int* d_slots = nullptr;
  int* h_slots = nullptr;  // pinned, kSlotRing x Bmax
  hipEvent_t slot_ev[4];
  int slot_i = 0;
  std::vector<int64_t> idx_tmp;

  // hipGraph replay of the fused step: two ping-pong instances, each with its
  // own pinned index buffer, so the host fills one while the other executes.
  struct GraphSlot {
    hipGraphExec_t exec = nullptr;
    int B = -1;
    const void* rb = nullptr;
    bool scaler = false;
    int* h_idx = nullptr;
    hipEvent_t done = nullptr;
  } gslot[2];
  int gcur = 0;
  // issue policy of the small-batch path (DDPG_GRAPH_AUTO):
  //   2 (default): always eager -- its 4 launches stream back to back, and a
  //     synchronous caller (the reference's worker) waits 86-87 us per step
  //     against 92-94 us for a graph replay (round 6, same box:
  //     profiles/r6/c2_issue_ab.txt; the graph launch costs more host time
  //     before the first kernel starts than the first eager launch);
  //   1: a step that finds the previous one finished replays the graph, a
  //     step issued while the previous is still running launches eagerly
  //     (the round-3..5 policy);
  //   0: always the graph.
  // Every policy issues the same kernels in the same order (bitwise equal
  // results); the large path always replays (the two measured equal there).
  int graph_auto = 2;
  hipEvent_t step_done = nullptr;
  bool use_graph = true;
  bool par = false;  // env DDPG_PAR=1: fork independent branches onto aux streams
  // small-batch fused path (small_batch.h): eligible dims, per-WG gradient slabs
  bool sb_ok = false;
  int sb_max_b = 0;
  float* sb_save = nullptr;   // per-row tensors the weight gradients read (SbSave)
  SbSave sb_sv{};
  SbGradTab sb_tab[2]{};      // weight-gradient tables: actor, critic
  float* sb_misc = nullptr;   // alpha[2] (of 4 floats)
  float* sb_whT = nullptr;    // [CH2][2 CH1] critic Wh^T shadow
  float* sb_w2T = nullptr;    // [AH2][AH1]   actor W2^T shadow
  bool sb_shadow_ok = false;  // cleared by every theta write outside the small path
  size_t sb_smem = 0;         // dynamic LDS bytes of the phase kernels
  unsigned* h_pred_done = nullptr;  // pinned coherent [SB_PRED_BLOCKS]: per-block completion seq
  unsigned pred_seq = 0;
  unsigned* h_stats_word = nullptr;  // pinned coherent: [0] completion word, then 2 floats
  unsigned stats_seq = 0;
  unsigned* h_rows_word = nullptr;  // pinned coherent: [0] completion word, floats from [16]
  unsigned rows_seq = 0;
  float* h_pred = nullptr;    // pinned [Bmax][A]: action-selection output (written by the GPU)
  int td_nqt = 0;      // fused step: target-critic partials pending in qpart_t for critic_loss
  int sb_xstride = 0;  // XCD packing of the phase kernels: 0 auto (on up to 32 workgroups),
                       // env DDPG_SB_XCD=1 always (8), =0 never (1)

  // kernel-path switches, read from the environment at ddpg_create (each is
  // exercised by tests/test_gpu_switches.py)
  struct {
    bool gemm_h = true;    // DDPG_GEMM_H=0: no bf16-twin GEMM (gemm_s3 NP=3 instead)
    bool gemm_s3 = true;   // DDPG_GEMM=f32: the fp32-input MFMA kernel for every GEMM
    bool thin_k = true;    // DDPG_THINK=0: the K <= 64 layers on the GEMMs
    bool gemm_h3 = true;   // DDPG_GEMM_H3=0: twin GEMMs with runtime slot addressing (gemm_h_kernel / gemm_h16_kernel)
    bool gemm_m16 = true;  // DDPG_GEMM_M16=0: fp32 contexts on the 32x32x16 gemm_h3_kernel instead of gemm_h3m_kernel
    bool nw_fuse = true;   // DDPG_NW_FUSE=0: dW1 / dWs / dWa on the skinny kernel instead of the dX epilogues
    int gemm256 = 0;       // DDPG_GEMM256=1: bf16 split-K weight gradients on gemm_h256.h (opt-in)
    bool gemm_hw = true;   // DDPG_GEMM_HW=0: bf16 weight gradients on gemm_h16_kernel instead of gemm_hw.h
    int xcd = 1;           // DDPG_XCD=0: no XCD-aware tile order
    bool xcd_rect = true;  // DDPG_XCD_RECT=0: row-major XCD runs only
    bool skinny = true;    // DDPG_SKINNY=0: skinny weight gradients on the GEMMs
    bool l1_batch = true;  // DDPG_L1BATCH=0: the step's first layers per network
    bool act_planes = true;  // DDPG_ACT32=1: fp32 copies of h1 / cat / cat2 as well
    bool slots_h2d = false;  // DDPG_SLOTS_H2D=1: upload the step's slots instead of reading them in place
    int tk_rpb = 0;          // DDPG_TK_RPB=n: thin_k row tiles per block (0: auto)
    bool kcomb = true;       // DDPG_KCOMB=0: no in-launch K split for small-M plain twin GEMMs
    int kc_blocks = 200;     // DDPG_KCOMB_BLOCKS=n: split plain twin GEMMs of fewer tiles
    bool prof_shapes = false;  // DDPG_PROF_SHAPES=1: GEMM / thin_k profile keys carry shapes
    bool skinny_nl = true;   // DDPG_SKINNY_NL=0: skinny kernel reads narrow rows by scalar loads
    bool half_twin = true;   // DDPG_HALF_TWIN=0: bf16 config stores cat2 / dcat state halves in fp32 too
    bool gemm_pack = true;   // DDPG_GEMM_PACK=0: deferred GEMMs launched one by one
    bool fwd_pack = true;    // DDPG_FWD_PACK=0: the step's forward layers in sequence
    bool stats_spin = true;  // DDPG_STATS_SPIN=0: stats read back by a copy + hipStreamSynchronize
    bool pred_spin = true;   // DDPG_PRED_SPIN=0: action selection waits with hipStreamSynchronize
    bool gather16 = true;    // DDPG_GATHER16=0: the one-row-per-wave gather everywhere
    bool tk_fwd = true;      // DDPG_TK_FWD=0: thin_k's generic epilogue for forward parts too
    int kc_splits = 4;       // DDPG_KCOMB_SPLITS=s: at most s splits per tile (2 .. KC_MAXS)
    bool kc_wgrad = true;    // DDPG_KCOMB_WGRAD=0: data-parallel weight gradients keep their slabs
  } sw;

  // small-M plan (ksplit_combine, gemm_common.h): kc_rot rotating partial
  // buffers of kc_part_n floats and ticket segments of kKcTickets, one per
  // combined launch in issue order (launches that may run concurrently on the
  // step's streams never share one)
  float* kc_part = nullptr;
  size_t kc_part_n = 0;
  unsigned* kc_ticket = nullptr;
  int kc_rot = 0, kc_next = 0;
  int gemm_defer = 0;  // > 0: gemm_launch queues gemm_h16i GEMMs for gemm_flush
  std::vector<DeferredGemm> deferred;
  int tk_slots = 512;  // thin_k blocks resident at once (ddpg_create: CUs x blocks per CU)

  // comm: every collective of the ctx is issued on cs (one stream, so the
  // communicator sees them in the same order on every rank); cs forks from the
  // producing stream and joins the consumer through the cev events
  ncclComm_t comm = nullptr;
  int world = 1, rank = 0;
  int cworld = 1;  // ranks in the communicator (1 for a 1-rank or a proxy communicator)
  int crank = 0;   // this rank in the communicator (0 for a proxy communicator)
  // the step graph captures the collectives too (env DDPG_GRAPH_COMM=0: such
  // steps stay eager); cleared if a capture with RCCL calls fails
  bool comm_graph = true;
  // learner steps run as a graph replay / eagerly (ddpg_step_counts)
  long long n_graph_steps = 0, n_eager_steps = 0;
  int graph_fail = 0;  // a capture with RCCL calls failed on this ctx
  hipStream_t cs = nullptr;
  hipEvent_t cev[8] = {};
  std::vector<int> win_open;  // profiling: open exchange-overlap windows (prof_recs indices)
  int test_cs_spin = 0;  // env DDPG_TEST_CS_SPIN=us (test hook, cs_spin_scale_kernel)

  // profiling
  bool prof = false;
  std::vector<ProfRec> prof_recs;
  std::vector<hipEvent_t> ev_pool;
  std::map<std::string, ProfAgg> prof_agg;
};

static constexpr int kSlotRing = 4;
static constexpr int kKcTickets = 1024;  // ticket segment (output tiles) per combined launch
static constexpr int kHeadRows = 64, kHeadRows4 = 32;

// ---------------------------------------------------------------- profiling helpers
static hipEvent_t ev_get(ddpg_ctx* c) {
  if (!c->ev_pool.empty()) {
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  HIP_TRY(hipEventCreate(&e));
  return e;
}

struct ProfScope {
  ddpg_ctx* c;
  size_t idx = (size_t)-1;
  ProfScope(ddpg_ctx* ctx, const char* name, double flops, double bytes) : c(ctx) {
    if (!c->prof) return;
    ProfRec rec{name, ev_get(c), ev_get(c), flops, bytes};
    HIP_TRY(hipEventRecord(rec.e0, c->cur));
    c->prof_recs.push_back(rec);
    idx = c->prof_recs.size() - 1;
  }
  ~ProfScope() {
    if (idx != (size_t)-1) (void)hipEventRecord(c->prof_recs[idx].e1, c->cur);
  }
};

// ---------------------------------------------------------------- GEMM launch
static GemmEpi epi_none() {
  GemmEpi e;
  memset(&e, 0, sizeof e);
  return e;
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

struct GemmPlan {
  int bm = 128, bn = 128, splits = 1, kps = 0;
  bool direct = false;  // the result went straight to the caller's `direct` buffer
  int mt(int M) const { return ceil_div(M, bm); }
  int nt(int N) const { return ceil_div(N, bn); }
};

// ---------------------------------------------------------------- bf16 twins
struct Twin {
  __bf16* p = nullptr;
  long long ps = 0;  // plane stride (elements)
};

enum { ACT_H1, ACT_CAT, ACT_CAT2 };
// ====================================================================== building blocks
static const float* P(ddpg_ctx* c, const float* base, const Tensor& t) { return base + t.off; }

template <class F>
static int guard(ddpg_ctx* c, F&& f) {
  try {
    f();
    return DDPG_OK;
  } catch (const DdpgError& e) {
    if (c) c->err = e.msg;
    g_err = e.msg;
    return e.code;
  } catch (const std::exception& e) {
    if (c) c->err = e.what();
    g_err = e.what();
    return DDPG_ENOMEM;
  }
}

template <class F>
static int rguard(ddpg_replay* rb, F&& f) {
  try {
    f();
    return DDPG_OK;
  } catch (const DdpgError& e) {
    if (rb) rb->err = e.msg;
    g_err = e.msg;
    return e.code;
  } catch (const std::exception& e) {
    if (rb) rb->err = e.what();
    g_err = e.what();
    return DDPG_ENOMEM;
  }
}

// deque position -> ring slot (deque holds insertions [total-count, total))
static inline int pos_to_slot(const ddpg_replay* rb, int64_t pos) {
  return (int)((rb->total - rb->count + pos) % rb->cap);
}


// ====================================================================== cross-unit functions
// gemm.hip
void gemm_setup(ddpg_ctx* c);  // ddpg_create: split caps, small-M buffers, kernel attributes
GemmPlan make_plan(int M, int N, int K, int splits, int cap = 64, bool big = false);
Twin act_twin(const ddpg_ctx* c, const float* q);
Twin operand_twin(const ddpg_ctx* c, const float* q);
template <int AL, int BL>
bool gemm_h_ok(const ddpg_ctx* c, const float* A, int lda, const float* B, int ldb, int M, int N,
               int K, int splits, int* Kh);
template <int AL, int BL>
GemmPlan gemm_launch(ddpg_ctx* c, const char* name, const float* A, int lda, const float* B,
                     int ldb, int M, int N, int K, const GemmEpi& e, int splits = 1, int cap = 64,
                     float* direct = nullptr);
TkPart tk_part(const float* X, int ldx, int K, const float* W, int ldw, int w_nk, int N,
               const float* bias, int act, float* out, int ldo);
int thin_k_launch(ddpg_ctx* c, const char* name, const TkPart* parts, int nparts, int M,
                  bool* dw_done = nullptr);
void gemm_flush(ddpg_ctx* c);
GemmPlan wgrad_launch(ddpg_ctx* c, const float* A, int lda, const float* B, int ldb, int M, int N,
                      int K, float* slab, int cap, float* direct);
// step.hip
void sb_setup(ddpg_ctx* c);  // ddpg_create: small-batch path eligibility and buffers
// dp.hip
void allreduce_on_cs(ddpg_ctx* c, int ev, const char* name, float* b0, size_t n0,
                     float* b1 = nullptr, size_t n1 = 0, bool with_stats = false,
                     const char* window = nullptr);
void stats_allreduce_on_cs(ddpg_ctx* c, bool gathered = false);
void join_cs(ddpg_ctx* c, int ev);
