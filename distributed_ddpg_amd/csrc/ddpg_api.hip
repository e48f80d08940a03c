// C-ABI implementation of the MI355X-native DDPG learner hot path.
// See include/ddpg_hip.h for the boundary and the reference interfaces each
// entry point replaces; DESIGN.md for the data layout and kernel list.
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
#include "gemm_f32.h"
#include "gemm_bf16.h"
#include "gemm_s3.h"
#include "gemm_h.h"
#include "gemm_h256.h"
#include "gemm_h3.h"
#include "thin_k.h"
#include "skinny.h"
#include "kernels.h"
#include "sampler.h"
#include "small_batch.h"

using namespace ddpg;

// ====================================================================== errors
static thread_local std::string g_err;

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
  explicit ddpg_replay(int64_t seed) : sampler(seed) {}
  size_t es() const { return f64 ? 8 : 4; }  // bytes per s / s2 / r element
  unsigned char* ps() const { return f64 ? (unsigned char*)rsd : (unsigned char*)rs; }
  unsigned char* ps2() const { return f64 ? (unsigned char*)rs2d : (unsigned char*)rs2; }
  unsigned char* pr() const { return f64 ? (unsigned char*)rrd : (unsigned char*)rr; }
};

static void replay_flush(ddpg_replay* rb);

// ====================================================================== context
struct ddpg_ctx {
  ddpg_cfg cfg{};
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
  // issue policy of the small-batch path (DDPG_GRAPH_AUTO=0: always the
  // graph): a step that finds the previous one finished (a caller that
  // synchronises every step, as the reference's worker does) replays the
  // graph -- the lower latency; a step issued while the previous is still
  // running (a pipelined caller) is launched eagerly -- the higher throughput
  // (its 4 launches stream back to back, where a graph launch stalls the queue
  // at its boundary: C2 +4 % same box; at large B the two measured equal, so
  // the large path always replays).  Both issue the same kernels in the same
  // order (bitwise equal results).
  bool graph_auto = true;
  hipEvent_t step_done = nullptr;
  bool use_graph = true;
  bool par = false;  // env DDPG_PAR=1: fork independent branches onto aux streams
  // small-batch fused path (small_batch.h): eligible dims, per-WG gradient slabs
  bool sb_ok = false;
  int sb_max_b = 0;
  float* sb_save = nullptr;   // per-row tensors the weight gradients read (SbSave)
  SbSave sb_sv{};
  SbGradTab sb_tab[2]{};      // weight-gradient tables: actor, critic
  float* sb_misc = nullptr;   // alpha[2] | stat_part[2 * G]
  float* sb_whT = nullptr;    // [CH2][2 CH1] critic Wh^T shadow
  float* sb_w2T = nullptr;    // [AH2][AH1]   actor W2^T shadow
  bool sb_shadow_ok = false;  // cleared by every theta write outside the small path
  size_t sb_smem = 0;         // dynamic LDS bytes of the phase kernels
  float* h_pred = nullptr;    // pinned [Bmax][A]: action-selection output (written by the GPU)
  int td_nqt = 0;      // fused step: target-critic partials pending in qpart_t for critic_loss
  int sb_xstride = 0;  // XCD packing of the phase kernels: 0 auto (on up to 32 workgroups),
                       // env DDPG_SB_XCD=1 always (8), =0 never (1)
  unsigned long long* sb_stamps = nullptr;  // diagnostic (env DDPG_SB_STAMPS=1)

  // kernel-path switches, read from the environment at ddpg_create (each is
  // exercised by tests/test_gpu_switches.py)
  struct {
    bool gemm_h = true;    // DDPG_GEMM_H=0: no bf16-twin GEMM (gemm_s3 NP=3 instead)
    bool gemm_s3 = true;   // DDPG_GEMM=f32: the fp32-input MFMA kernel for every GEMM
    bool thin_k = true;    // DDPG_THINK=0: the K <= 64 layers on the GEMMs
    int gemm_mf = 16;      // DDPG_GEMM_MF=32: bf16 config on the 32x32x16 twin GEMM
    bool gemm_h3 = true;   // DDPG_GEMM_H3=0: twin GEMMs with runtime slot addressing (gemm_h_kernel / gemm_h16_kernel)
    int gemm256 = 0;       // DDPG_GEMM256=1 / 4: bf16 split-K weight gradients on gemm_h256.h; 2, 3: more shapes
    int xcd = 1;           // DDPG_XCD=0: no XCD-aware tile order
    bool xcd_rect = true;  // DDPG_XCD_RECT=0: row-major XCD runs only
    bool skinny = true;    // DDPG_SKINNY=0: skinny weight gradients on the GEMMs
    bool l1_batch = true;  // DDPG_L1BATCH=0: the step's first layers per network
    bool act_planes = true;  // DDPG_ACT32=1: fp32 copies of h1 / cat / cat2 as well
    bool slots_h2d = false;  // DDPG_SLOTS_H2D=1: upload the step's slots instead of reading them in place
    int tk_rpb = 0;          // DDPG_TK_RPB=n: thin_k row tiles per block (0: auto)
    bool kcomb = true;       // DDPG_KCOMB=0: no in-launch K split for small-M plain twin GEMMs
    int kc_blocks = 200;     // DDPG_KCOMB_BLOCKS=n: split plain twin GEMMs of fewer tiles
  } sw;

  // small-M plan (ksplit_combine, gemm_common.h): kc_rot rotating partial
  // buffers of kc_part_n floats and ticket segments of kKcTickets, one per
  // combined launch in issue order (launches that may run concurrently on the
  // step's streams never share one)
  float* kc_part = nullptr;
  size_t kc_part_n = 0;
  unsigned* kc_ticket = nullptr;
  int kc_rot = 0, kc_next = 0;

  // comm: every collective of the ctx is issued on cs (one stream, so the
  // communicator sees them in the same order on every rank); cs forks from the
  // producing stream and joins the consumer through the cev events
  ncclComm_t comm = nullptr;
  int world = 1, rank = 0;
  int cworld = 1;  // ranks in the communicator (1 for a 1-rank or a proxy communicator)
  // the step graph captures the collectives too (env DDPG_GRAPH_COMM=0: such
  // steps stay eager); cleared if a capture with RCCL calls fails
  bool comm_graph = true;
  hipStream_t cs = nullptr;
  hipEvent_t cev[8] = {};
  int win_rec = -1;     // profiling: open exchange-overlap window (prof_recs index)
  int test_cs_spin = 0;  // env DDPG_TEST_CS_SPIN=us (test hook, cs_spin_scale_kernel)

  // profiling
  bool prof = false;
  std::vector<ProfRec> prof_recs;
  std::vector<hipEvent_t> ev_pool;
  std::map<std::string, ProfAgg> prof_agg;
};

static constexpr int kSlotRing = 4;
static constexpr int kKcTickets = 1024;  // ticket segment (output tiles) per combined launch
static constexpr int kHeadRows = 64, kHeadRows4 = 64;

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

static void prof_collect(ddpg_ctx* c) {
  if (c->prof_recs.empty()) return;
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (auto st : c->aux) HIP_TRY(hipStreamSynchronize(st));
  if (c->cs) HIP_TRY(hipStreamSynchronize(c->cs));
  for (auto& r : c->prof_recs) {
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, r.e0, r.e1));
    ProfAgg& a = c->prof_agg[r.name];
    a.ms += ms;
    a.flops += r.flops;
    a.bytes += r.bytes;
    a.launches += 1;
    c->ev_pool.push_back(r.e0);
    c->ev_pool.push_back(r.e1);
  }
  c->prof_recs.clear();
}

// ---------------------------------------------------------------- GEMM launch
static GemmEpi epi_none() {
  GemmEpi e;
  memset(&e, 0, sizeof e);
  return e;
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Block-count target for tile selection (env DDPG_GEMM_MIN_BLOCKS overrides).
static int g_min_blocks = 1024;

struct GemmPlan {
  int bm = 128, bn = 128, splits = 1, kps = 0;
  bool direct = false;  // the result went straight to the caller's `direct` buffer
  int mt(int M) const { return ceil_div(M, bm); }
  int nt(int N) const { return ceil_div(N, bn); }
};

static const int kTiles[4][2] = {{128, 128}, {128, 64}, {64, 128}, {64, 64}};

// Largest tile (no more than one 64-row/col of padding) whose grid reaches
// the block target; otherwise the one with the most blocks.
static void pick_tile(int M, int N, int min_blocks, int* bm, int* bn) {
  int best = -1, best_blocks = -1;
  for (int t = 0; t < 4; ++t) {
    const int tm = kTiles[t][0], tn = kTiles[t][1];
    if (tm > 64 && M <= 64) continue;
    if (tn > 64 && N <= 64) continue;
    const int blocks = ceil_div(M, tm) * ceil_div(N, tn);
    if (blocks >= min_blocks) {
      *bm = tm;
      *bn = tn;
      return;
    }
    if (blocks > best_blocks) {
      best_blocks = blocks;
      best = t;
    }
  }
  *bm = kTiles[best][0];
  *bn = kTiles[best][1];
}

// Plan for a plain (splits = 1) GEMM or a split-K weight-gradient GEMM
// (splits = 0: auto, ~512 blocks, >= 128 k per split, <= cap).
static GemmPlan make_plan(int M, int N, int K, int splits, int cap = 64, bool big = false) {
  GemmPlan p;
  if (big) {  // bf16 kernel: fixed 128 x 128 tile
    p.bm = p.bn = 128;
    if (splits != 1) {
      const int tiles = ceil_div(M, 128) * ceil_div(N, 128);
      splits = std::max(1, 512 / tiles);
      splits = std::min(splits, std::max(1, K / 128));
      splits = std::min(splits, cap);
    }
  } else if (splits == 1) {
    pick_tile(M, N, g_min_blocks, &p.bm, &p.bn);
  } else {
    p.bm = M <= 64 ? 64 : 128;
    p.bn = N <= 64 ? 64 : 128;
    const int tiles = ceil_div(M, p.bm) * ceil_div(N, p.bn);
    splits = std::max(1, 512 / tiles);
    splits = std::min(splits, std::max(1, K / 128));
    splits = std::min(splits, cap);
  }
  p.kps = rup(std::max(1, ceil_div(K, splits)), GBK);
  p.splits = std::max(1, ceil_div(K, p.kps));
  return p;
}

// ---------------------------------------------------------------- bf16 twins
struct Twin {
  __bf16* p = nullptr;
  long long ps = 0;  // plane stride (elements)
};

// Twin of an activation buffer element (nullptr unless the buffer is twinned)
static Twin act_twin(const ddpg_ctx* c, const float* q) {
  Twin t;
  if (!c->hnp || !q) return t;
  for (const auto& b : c->twinned)
    if (q >= b.first && q < b.first + b.second) {
      t.p = c->atw + (q - c->dact);
      t.ps = (long long)c->act_n;
      return t;
    }
  return t;
}

enum { ACT_H1, ACT_CAT, ACT_CAT2 };
static bool gemm_h_ok_fwd_l2(ddpg_ctx* c, int which, int B);  // below

// fp32 contexts: an activation whose every reader takes its three exact bf16
// planes (the twin GEMMs, and the EluGrad factor of the next backward GEMM's
// epilogue, `GemmEpi::auxh`) is written as planes only -- 4 B per element
// less to write for 2 B more to read.  h1 (actor layer 1), cat (critic layer
// 1, train / predict) and cat2 (critic layer 1 at (s, mu)).  DDPG_ACT32=1
// keeps the fp32 copies.
static bool act_planes_only(ddpg_ctx* c, int which, int B) {
  if (c->hnp != 3 || !c->sw.act_planes) return false;
  const float* q = which == ACT_H1 ? c->h1 : which == ACT_CAT ? c->cat : c->cat2;
  if (!act_twin(c, q).p) return false;
  return gemm_h_ok_fwd_l2(c, which, B);
}

// Twin of a GEMM operand: a parameter (theta / target, while the parameter
// twins are current) or a twinned activation buffer
static Twin operand_twin(const ddpg_ctx* c, const float* q) {
  Twin t;
  if (!c->hnp || !q) return t;
  const size_t PT = c->L.total;
  if (c->wtw_ok) {
    if (q >= c->theta && q < c->theta + PT) {
      t.p = c->wtw + (q - c->theta);
      t.ps = (long long)PT;
      return t;
    }
    if (q >= c->target && q < c->target + PT) {
      t.p = c->wtw + (size_t)c->hnp * PT + (q - c->target);
      t.ps = (long long)PT;
      return t;
    }
  }
  return act_twin(c, q);
}

// Row buffers whose columns past the logical width are always zero (their
// writers touch only the first S / A columns): a contraction over them may run
// K-padded to its kernel's k step, the padded products being exact zeros.
static bool zero_padded(const ddpg_ctx* c, const float* q) {
  return q == c->s || q == c->s2 || q == c->a || q == c->ta2 || q == c->mu || q == c->dz3;
}

// Rebuild the parameter twins after a write that bypassed Adam / the soft
// update (set_params, checkpoint restore, the small-batch path).  Eager:
// never inside a captured step (the step's own Adam / soft-update launches
// keep them current).
static void twins_refresh(ddpg_ctx* c) {
  if (!c->hnp || c->wtw_ok) return;
  const size_t PT = c->L.total;
  hipLaunchKernelGGL(twin_kernel, dim3(2048), dim3(256), 0, c->stream, c->theta, (long long)PT,
                     c->wtw, (long long)PT, c->hnp);
  hipLaunchKernelGGL(twin_kernel, dim3(2048), dim3(256), 0, c->stream, c->target, (long long)PT,
                     c->wtw + (size_t)c->hnp * PT, (long long)PT, c->hnp);
  HIP_TRY(hipGetLastError());
  c->wtw_ok = true;
}


template <int AL, int BL, int VA, int VB>
static void gemm_dispatch(const GemmPlan& p, dim3 grid, hipStream_t st, const GemmArgs& g) {
  if (p.bm == 128 && p.bn == 128)
    hipLaunchKernelGGL((gemm_f32_kernel<AL, BL, VA, VB, 128, 128>), grid, dim3(GNT), 0, st, g);
  else if (p.bm == 128)
    hipLaunchKernelGGL((gemm_f32_kernel<AL, BL, VA, VB, 128, 64>), grid, dim3(GNT), 0, st, g);
  else if (p.bn == 128)
    hipLaunchKernelGGL((gemm_f32_kernel<AL, BL, VA, VB, 64, 128>), grid, dim3(GNT), 0, st, g);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<AL, BL, VA, VB, 64, 64>), grid, dim3(GNT), 0, st, g);
}

// XCD tile order for an nx x ny grid of BM x BN tiles (xcd_tile): the
// rectangle of tiles per XCD with the fewest operand-panel bytes
// (H row panels of BM rows + W column panels of BN columns), when 8 such
// rectangles tile the grid and it reads fewer bytes than the row-major runs.  env DDPG_XCD_RECT=0
// keeps the runs.
static int xcd_rect(const ddpg_ctx* c, int nx, int ny, int BM, int BN) {
  const int on = c->sw.xcd;
  if (!on || !c->sw.xcd_rect || (nx * ny) % 8) return on;
  const int T = nx * ny / 8;
  int best = -1, best_cost = 0;
  for (int W = 1; W <= nx; ++W) {
    if (nx % W || T % W) continue;
    const int H = T / W;
    if (ny % H || (nx / W) * (ny / H) != 8) continue;
    const int cost = H * BM + W * BN;
    if (best < 0 || cost < best_cost) {
      best = W;
      best_cost = cost;
    }
  }
  // keep the row-major runs unless the rectangle reads strictly fewer bytes
  const int run_cost = T % nx ? -1 : (T / nx) * BM + nx * BN;
  if (best < 0 || (run_cost >= 0 && best_cost >= run_cost)) return on;
  return 16 + best;
}

static bool use_bf16(const ddpg_ctx* c, int M, int N, bool vec);
static bool use_s3(const ddpg_ctx* c, int M, int N, bool vec);

// Whether gemm_launch runs this GEMM on the bf16-twin kernel (both operands
// twinned, shapes in its tiles, K in whole k-tiles -- or K-padded first
// layers: A rows zero past K, B a parameter twin whose rows past K are the
// next tensors' finite values, multiplied by zero); *Kh = the K it runs.
// Producers use it to skip fp32 copies nobody reads.
template <int AL, int BL>
static bool gemm_h_ok(const ddpg_ctx* c, const float* A, int lda, const float* B, int ldb, int M,
                      int N, int K, int splits, int* Kh) {
  if (!(c->sw.gemm_h && c->hnp && M >= 128 && N >= 128 && N % 8 == 0 && lda % 8 == 0 &&
        ldb % 8 == 0 && (AL == L_RK || M % 8 == 0) && (BL == L_RK || N % 8 == 0)))
    return false;
  const int BKh = c->hnp == 1 ? 64 : 32;
  const Twin ta = operand_twin(c, A), tb = operand_twin(c, B);
  int k = K;
  if (K % BKh && AL == L_RK && BL == L_KR && zero_padded(c, A) && rup(K, BKh) <= lda && tb.p &&
      tb.ps == (long long)c->L.total && splits == 1)
    k = rup(K, BKh);
  if (!(k % BKh == 0 && ta.p && tb.p && aligned16(ta.p) && aligned16(tb.p))) return false;
  *Kh = k;
  return true;
}

// gemm_h256_kernel (bf16 configuration, 256 x 256 tiles): splits of a
// weight gradient -- about one block per CU, every split a whole number of
// the kernel's 4-step trips (kps % 128 == 0)
static int h256_splits(int M, int N, int K, int cap) {
  const int tiles = (M / H2_BM) * (N / H2_BN);
  int sp = std::max(1, 256 / tiles);
  sp = std::min(std::min(sp, cap), std::max(1, K / 128));
  while (sp > 1 && (K % sp || (K / sp) % 128)) --sp;
  return sp;
}
// -1: not taken; 0: split-K weight gradient with a plain slab epilogue
// (DDPG_GEMM256=1); 1 / 2: unsplit GEMMs (=2 / =3).  Full tiles only.  Off by
// default: in the C5 step the finer split's extra slab reduction cost more
// than the faster main loop saved (profiles/r3/gemm_h256_ab_c5.txt).
static int h256_mode(const ddpg_ctx* c, int M, int N, int Kh, int splits, const GemmEpi& e,
                     bool dx_layout, bool a_rk) {
  if (!(c->hnp == 1 && c->sw.gemm256 && c->sw.gemm_mf == 16 && M % H2_BM == 0 &&
        N % H2_BN == 0 && Kh % 128 == 0))
    return -1;
  const bool plain = !e.bias && e.act == 0 && e.post == 0 && !e.colsum && !e.proj_out && !e.outh;
  if (splits != 1) return plain ? 0 : -1;
  // measurement switches (same-box A/B): DDPG_GEMM256=2 adds the
  // >= 256-tile dX GEMMs (MODE 1); 3 also every unsplit GEMM of >= 128 tiles
  // (MODE 2, relying on the step's concurrent streams to fill the chip)
  const bool dx = !e.bias && e.act == 0 && e.post == 1;
  const int tiles = (M / H2_BM) * (N / H2_BN);
  if ((c->sw.gemm256 == 2 || c->sw.gemm256 == 3) && dx && dx_layout && tiles >= 256) return 1;
  return c->sw.gemm256 == 3 && a_rk && tiles >= 128 ? 2 : -1;
}

// direct: for a split-K weight gradient, where to write the result when the
// plan ends up with one split (no slab, no reduction; plan.direct = true).
template <int AL, int BL>
static GemmPlan gemm_launch(ddpg_ctx* c, const char* name, const float* A, int lda,
                            const float* B, int ldb, int M, int N, int K, const GemmEpi& e,
                            int splits = 1, int cap = 64, float* direct = nullptr) {
  const int contA = (AL == L_RK) ? K : M;
  const int contB = (BL == L_RK) ? K : N;
  const bool va = (contA % 4 == 0) && (lda % 4 == 0) && aligned16(A);
  const bool vb = (contB % 4 == 0) && (ldb % 4 == 0) && aligned16(B);
  const bool vec = va && vb;
  const bool bf = use_bf16(c, M, N, vec);
  const bool s3 = !bf && use_s3(c, M, N, vec);
  GemmPlan p = make_plan(M, N, K, splits, cap, bf || s3);
  if (M <= 0 || N <= 0) return p;
  {  // the element-wise combinations gemm_epilogue is specialised on
    const bool b = e.bias != nullptr;
    const bool ok = (!b && e.act == 0 && e.post == 0) || (b && e.act == 1 && e.post == 0) ||
                    (b && e.act == 1 && e.post == 2) || (!b && e.act == 0 && e.post == 1) ||
                    (b && e.act == 0 && e.post == 0);
    if (!ok) throw einval("gemm %s: unsupported epilogue (bias %d act %d post %d)", name, b, e.act,
                          e.post);
  }
  // a twinned output gets its bf16 twin written by the epilogue
  GemmEpi ee = e;
  if (!ee.outh && ee.out && !ee.out_split_stride) {
    const Twin to = act_twin(c, ee.out);
    if (to.p) {
      ee.outh = to.p;
      ee.h_plane_stride = to.ps;
      ee.h_planes = c->hnp;
    }
  }
  // bf16-twin operands (gemm_h.h): both operands twinned, K in whole k-tiles
  int Kh = 0;
  if (gemm_h_ok<AL, BL>(c, A, lda, B, ldb, M, N, K, splits, &Kh)) {
    const int BKh = c->hnp == 1 ? 64 : 32, BMh = c->hnp == 1 ? 256 : 128;
    const Twin ta = operand_twin(c, A), tb = operand_twin(c, B);
    {
      // as requested (the 256 x 128 plan below rewrites both)
      const int splits_req = splits;  // 1: plain GEMM; otherwise a split-K weight gradient
      const GemmEpi ee_req = ee;
      GemmPlan h;
      h.bm = BMh;
      h.bn = HG_BN;
      if (splits != 1) {  // ~one block per CU (144 KB of LDS each)
        const int tiles = ceil_div(M, BMh) * ceil_div(N, HG_BN);
        splits = std::max(1, 256 / tiles);
        splits = std::min(splits, std::max(1, K / (4 * BKh)));
        splits = std::min(splits, cap);
      }
      h.kps = rup(ceil_div(Kh, std::max(1, splits)), BKh);
      h.splits = ceil_div(Kh, h.kps);
      if (h.splits == 1 && direct) {
        ee.out = direct;
        ee.out_split_stride = 0;
        h.direct = true;
      }
      GemmHArgs a;
      // small-M plan: a plain GEMM (forward / dX) whose tiles leave most CUs
      // idle -- per-rank batches of a strong-scaling run, e.g. C3 at B = 512
      // has 32 forward tiles for 256 CUs -- splits K over ~256 blocks (>= 3
      // k-tiles each) and combines the splits in-launch before its epilogue
      // (ksplit_combine).  The immediate-offset kernels only.
      const bool kc_kernel = c->sw.gemm_h3 && (c->hnp == 3 || (c->hnp == 1 && c->sw.gemm_mf == 16 &&
                                                              AL == L_RK));
      if (splits_req == 1 && kc_kernel && c->kc_part) {
        const int tiles = h.nt(N) * h.mt(M);
        const int nkt = Kh / BKh;
        int sk = std::min(ceil_div(256, tiles), nkt / 3);
        if (tiles < c->sw.kc_blocks && sk >= 2) {
          const int kps = ceil_div(nkt, sk) * BKh;
          sk = ceil_div(Kh, kps);
          if (sk >= 2 && (size_t)sk * tiles * BMh * HG_BN <= c->kc_part_n && tiles <= kKcTickets) {
            const int slot = c->kc_next++ % c->kc_rot;
            a.kpart = c->kc_part + (size_t)slot * c->kc_part_n;
            a.kticket = c->kc_ticket + (size_t)slot * kKcTickets;
            h.kps = kps;
            h.splits = sk;
          }
        }
      }
      a.A = ta.p;
      a.B = tb.p;
      a.pa = ta.ps;
      a.pb = tb.ps;
      a.M = M;
      a.N = N;
      a.K = Kh;
      a.lda = lda;
      a.ldb = ldb;
      a.kps = h.kps;
      a.xcd = xcd_rect(c, h.nt(N), h.mt(M), BMh, HG_BN);
      a.e = ee;
      static const char* lay[2] = {"RK", "KR"};
      // bf16 configuration, whole 256 x 256 tiles (gemm_h256.h): the split-K
      // weight gradients (plain slabs, MODE 0) and the dX GEMMs whose grid
      // fills the chip unsplit (>= 256 tiles, MODE 1)
      const int mode256 =
          h256_mode(c, M, N, Kh, splits_req, ee_req, AL == L_RK && BL == L_RK, AL == L_RK);
      if (mode256 >= 0) {
        GemmPlan q;
        q.bm = q.bn = H2_BM;
        int sp = mode256 == 0 ? h256_splits(M, N, Kh, cap) : 1;
        // DDPG_GEMM256=4: the 256 x 128 plan's split count (no extra slab to
        // reduce; half the blocks, beside the concurrent dX chain)
        if (mode256 == 0 && c->sw.gemm256 == 4 && Kh % h.splits == 0 && (Kh / h.splits) % 128 == 0)
          sp = h.splits;
        q.kps = Kh / sp;
        q.splits = sp;
        GemmEpi e2 = ee_req;
        if (q.splits == 1 && direct) {
          e2.out = direct;
          e2.out_split_stride = 0;
          q.direct = true;
        }
        a.e = e2;
        a.kps = q.kps;
        a.xcd = xcd_rect(c, q.nt(N), q.mt(M), H2_BM, H2_BN);
        char key[112];
        snprintf(key, sizeof key, "gemm_h256_kernel<%s,%s,MODE=%d>|%s", lay[AL], lay[BL], mode256,
                 name);
        ProfScope ps(c, key, 2.0 * M * N * (double)K,
                     2.0 * ((double)M * K + (double)K * N) + 4.0 * (double)M * N * q.splits);
        const dim3 grid(q.nt(N), q.mt(M), q.splits);
        if (mode256 == 0) {
          hipLaunchKernelGGL((gemm_h256_kernel<AL, BL, 0>), grid, dim3(H2_NT), 0, c->cur, a);
        } else if (mode256 == 2) {
          if constexpr (AL == L_RK)
            hipLaunchKernelGGL((gemm_h256_kernel<AL, BL, 2>), grid, dim3(H2_NT), 0, c->cur, a);
        } else if constexpr (AL == L_RK && BL == L_RK) {
          hipLaunchKernelGGL((gemm_h256_kernel<AL, BL, 1>), grid, dim3(H2_NT), 0, c->cur, a);
        }
        HIP_TRY(hipGetLastError());
        return q;
      }
      // bf16 configuration: the 16x16x32-MFMA kernel (DDPG_GEMM_MF=32 keeps 32x32x16)
      const bool h16 = c->hnp == 1 && c->sw.gemm_mf == 16;
      char key[112];
      // "/kc": the splits are combined in-launch (small-M plan)
      snprintf(key, sizeof key, "%s<%s,%s,NP=%d>|%s%s",
               h16 ? (AL == L_RK && c->sw.gemm_h3 ? "gemm_h16i_kernel" : "gemm_h16_kernel")
                   : (c->hnp == 3 && c->sw.gemm_h3) ? "gemm_h3_kernel" : "gemm_h_kernel",
               lay[AL], lay[BL], c->hnp, name, a.kpart ? "/kc" : "");
      ProfScope ps(c, key, 2.0 * M * N * (double)K,
                   2.0 * c->hnp * ((double)M * K + (double)K * N) +
                       4.0 * (double)M * N * h.splits);
      const dim3 grid(h.nt(N), h.mt(M), h.splits);
      if (h16 && AL == L_RK && c->sw.gemm_h3) {
        // immediate-offset addressing (gemm_h3.h), RK A operands
        if constexpr (AL == L_RK)
          hipLaunchKernelGGL((gemm_h16i_kernel<AL, BL>), grid, dim3(HG_NT), 0, c->cur, a);
      } else if (h16)
        hipLaunchKernelGGL((gemm_h16_kernel<AL, BL, 1, 256, 64>), grid, dim3(HG_NT), 0, c->cur, a);
      else if (c->hnp == 1)
        hipLaunchKernelGGL((gemm_h_kernel<AL, BL, 1, 256, 64>), grid, dim3(HG_NT), 0, c->cur, a);
      else if (c->sw.gemm_h3)
        // the same kernel with immediate-offset addressing (gemm_h3.h)
        hipLaunchKernelGGL((gemm_h3_kernel<AL, BL>), grid, dim3(HG_NT), 0, c->cur, a);
      else
        // SCH 1: fragment reads spread over the MFMA gaps (+2-4 % over the
        // burst schedule, bitwise equal; profiles/r3/gemmh_sched_c3.txt)
        hipLaunchKernelGGL((gemm_h_kernel<AL, BL, 3, 128, 32, 1>), grid, dim3(HG_NT), 0, c->cur, a);
      HIP_TRY(hipGetLastError());
      return h;
    }
  }
  if (p.splits == 1 && direct) {
    ee.out = direct;
    ee.out_split_stride = 0;
    p.direct = true;
  }
  GemmArgs g;
  g.A = A;
  g.B = B;
  g.M = M;
  g.N = N;
  g.K = K;
  g.lda = lda;
  g.ldb = ldb;
  g.kps = p.kps;
  g.xcd = c->sw.xcd;
  g.e = ee;
  dim3 grid(p.nt(N), p.mt(M), p.splits);
  // profile key "<kernel symbol>|<phase>": the symbol part matches rocprofv3's kernel names
  static const char* lay[2] = {"RK", "KR"};
  char key[112];
  if (bf || s3)  // one bf16 plane (bf16 configuration) or the exact three-plane split
    snprintf(key, sizeof key, "gemm_s3_kernel<%s,%s,NP=%d>|%s", lay[AL], lay[BL], bf ? 1 : 3,
             name);
  else
    snprintf(key, sizeof key, "gemm_f32_kernel<%s,%s,%d,%d,%d,%d>|%s", lay[AL], lay[BL],
             va ? 4 : 1, vb ? 4 : 1, p.bm, p.bn, name);
  // algorithmic bytes: each operand read once, the output (per split slab) written once
  ProfScope ps(c, key, 2.0 * M * N * (double)K,
               4.0 * ((double)M * K + (double)K * N + (double)M * N * p.splits));
  if (bf)
    hipLaunchKernelGGL((gemm_s3_kernel<AL, BL, 1>), grid, dim3(S3_NT), 0, c->cur, g);
  else if (s3)
    hipLaunchKernelGGL((gemm_s3_kernel<AL, BL, 3>), grid, dim3(S3_NT), 0, c->cur, g);
  else if (va && vb)
    gemm_dispatch<AL, BL, 4, 4>(p, grid, c->cur, g);
  else if (va)
    gemm_dispatch<AL, BL, 4, 1>(p, grid, c->cur, g);
  else if (vb)
    gemm_dispatch<AL, BL, 1, 4>(p, grid, c->cur, g);
  else
    gemm_dispatch<AL, BL, 1, 1>(p, grid, c->cur, g);
  HIP_TRY(hipGetLastError());
  return p;
}

// bf16 MFMA for the large GEMMs of a DDPG_BF16 context (thin / unaligned
// shapes stay on the exact-fp32 kernel)
static bool use_bf16(const ddpg_ctx* c, int M, int N, bool vec) {
  return c->cfg.dtype == DDPG_BF16 && vec && M >= 128 && N >= 128;
}

// fp32 contexts: the large GEMMs run fp32-accurate on the bf16 pipe
// (gemm_s3.h, three-plane split); env DDPG_GEMM=f32 keeps every GEMM on the
// fp32-input MFMA kernel.
static bool use_s3(const ddpg_ctx* c, int M, int N, bool vec) {
  return c->sw.gemm_s3 && c->cfg.dtype == DDPG_FP32 && vec && M >= 128 && N >= 128;
}

// Thin-K layers (thin_k.h) of fp32 contexts: K <= 64 and multiple of 8,
// 4-aligned widths / leading dims, 16-byte aligned operands (anything else goes
// through the GEMMs).  env DDPG_THINK=0 routes every such layer to the GEMMs.
static bool tk_valid(const TkPart& q) {
  // W[n][k] (w_nk) may have any stride: the kernel loads it as scalars then
  return q.K >= TK_KALIGN && q.K % TK_KALIGN == 0 && q.K <= TK_MAXK && q.ldx % 4 == 0 &&
         (q.w_nk || (q.ldw % 4 == 0 && aligned16(q.W))) && q.N % 4 == 0 && q.ldo % 4 == 0 &&
         aligned16(q.X) &&
         (!q.out || aligned16(q.out)) && (!q.bias || aligned16(q.bias)) &&
         (!q.aux || (q.ldaux % 4 == 0 && aligned16(q.aux)));
}

static TkPart tk_part(const float* X, int ldx, int K, const float* W, int ldw, int w_nk, int N,
                      const float* bias, int act, float* out, int ldo) {
  TkPart p;
  memset(&p, 0, sizeof p);
  p.X = X;
  p.ldx = ldx;
  p.K = K;
  p.W = W;
  p.ldw = ldw;
  p.w_nk = w_nk;
  p.N = N;
  p.bias = bias;
  p.act = act;
  p.out = out;
  p.ldo = ldo;
  return p;
}

// Launch 1 .. TK_MAXP thin-K parts over M rows; returns the number of 64-row
// blocks (the row count of colsum partials), or 0 (nothing launched) when a
// layer is not eligible and the caller must use the GEMM.
static int thin_k_launch(ddpg_ctx* c, const char* name, const TkPart* parts, int nparts, int M) {
  if (!c->sw.thin_k || nparts < 1 || nparts > TK_MAXP) return 0;
  TkPart pp[TK_MAXP];
  for (int i = 0; i < nparts; ++i) {
    pp[i] = parts[i];
    // K-padded to the 8-step of the kernel over zero-padded rows (the W rows
    // past K read are finite parameters of the next tensor, times zero)
    if (pp[i].K % TK_KALIGN && zero_padded(c, pp[i].X) && rup(pp[i].K, TK_KALIGN) <= pp[i].ldx &&
        pp[i].W >= c->dparams && pp[i].W < c->dparams + 2 * c->L.total)
      pp[i].K = rup(pp[i].K, TK_KALIGN);
    if (!tk_valid(pp[i])) return 0;
  }
  parts = pp;
  TkArgs a;
  memset(&a, 0, sizeof a);
  int nmax = 0;
  double flops = 0, bytes = 0;
  for (int i = 0; i < nparts; ++i) {
    a.p[i] = parts[i];
    const Twin to = act_twin(c, parts[i].out);
    if (to.p && !a.p[i].outh) {
      a.p[i].outh = to.p;
      a.p[i].hps = to.ps;
      a.p[i].hnp = c->hnp;
    }
    nmax = std::max(nmax, parts[i].N);
    flops += 2.0 * M * parts[i].N * (double)parts[i].K;
    bytes += 4.0 * ((double)M * parts[i].K + (double)parts[i].K * parts[i].N +
                    (double)M * parts[i].N);
  }
  a.M = M;
  const int mt = ceil_div(M, TK_ROWS);
  const int nc = ceil_div(nmax, TK_COLS);
  // row tiles per block: the fewest that keep the grid within one round of
  // the chip's block slots (256 CUs x 2 blocks of 72 KB LDS), so that a block
  // stages its W panel once for several row tiles and overlaps the next X
  // tile's loads with its stores (env DDPG_TK_RPB=n forces n; 1 = one tile)
  int rpb = 1;
  if (c->sw.tk_rpb > 0) {
    rpb = std::min(c->sw.tk_rpb, mt);
  } else {
    constexpr int kSlots = 256 * 2;
    while (rpb < mt && nc * nparts * ceil_div(mt, rpb) > kSlots) ++rpb;
  }
  a.mt = mt;
  a.rpb = rpb;
  char key[96];
  snprintf(key, sizeof key, "thin_k_kernel|%s", name);
  ProfScope ps(c, key, flops, bytes);
  hipLaunchKernelGGL(thin_k_kernel, dim3(nc, ceil_div(mt, rpb), nparts), dim3(TK_NT), 0, c->cur, a);
  HIP_TRY(hipGetLastError());
  return mt;
}

// ====================================================================== building blocks
static const float* P(ddpg_ctx* c, const float* base, const Tensor& t) { return base + t.off; }

// Every twin-GEMM reader of the activation `which` at batch B takes the twin
// (act_planes_only): h1 -> actor layer 2 and dW2; cat -> critic hidden layer
// and dWh; cat2 -> the critic hidden layer at (s, mu).
static bool gemm_h_ok_fwd_l2(ddpg_ctx* c, int which, int B) {
  const Layout& L = c->L;
  int kh;
  if (which == ACT_H1)
    return gemm_h_ok<L_RK, L_KR>(c, c->h1, c->ldAH1, P(c, c->theta, L.a[AW2]), c->AH2, B, c->AH2,
                                 c->AH1, 1, &kh) &&
           gemm_h_ok<L_KR, L_KR>(c, c->h1, c->ldAH1, c->dz2, c->ldAH2, c->AH1, c->AH2, B, 0, &kh);
  const float* q = which == ACT_CAT ? c->cat : c->cat2;
  const bool fwd = gemm_h_ok<L_RK, L_KR>(c, q, c->ldC, P(c, c->theta, L.c[CWH]), c->CH2, B,
                                         c->CH2, 2 * c->CH1, 1, &kh);
  if (which == ACT_CAT2) return fwd;
  return fwd && gemm_h_ok<L_KR, L_KR>(c, c->cat, c->ldC, c->dhp, c->ldCH2, 2 * c->CH1, c->CH2, B,
                                      0, &kh);
}

// The EluGrad operand of a post-1 epilogue: the fp32 activation, or its planes
// when only those were written.
static void epi_aux(ddpg_ctx* c, GemmEpi& e, int which, int B, const float* q, int ld) {
  e.ldaux = ld;
  if (act_planes_only(c, which, B)) {
    const Twin t = act_twin(c, q);
    e.aux = nullptr;
    e.auxh = t.p;
    e.auxh_ps = t.ps;
  } else {
    e.aux = q;
  }
}

// The actor's first layer as a thin-K part.  The target path's h1 is read only
// by the next layer: when that runs on the twin GEMM, only the twin is written.
static TkPart actor_l1_part(ddpg_ctx* c, const float* base, const float* s, int B, float* h1,
                            Twin* twin) {
  const Layout& L = c->L;
  int kh;
  const bool planes = (h1 == c->th1 && gemm_h_ok<L_RK, L_KR>(c, h1, c->ldAH1,
                                                             P(c, base, L.a[AW2]), c->AH2, B,
                                                             c->AH2, c->AH1, 1, &kh)) ||
                      (h1 == c->h1 && act_planes_only(c, ACT_H1, B));
  const Twin h1t = planes ? act_twin(c, h1) : Twin();
  TkPart tp = tk_part(s, c->ldS, c->S, P(c, base, L.a[AW1]), c->AH1, 0, c->AH1,
                      P(c, base, L.a[AB1]), 1, h1t.p ? nullptr : h1, c->ldAH1);
  tp.outh = h1t.p;
  tp.hps = h1t.ps;
  tp.hnp = c->hnp;
  if (twin) *twin = h1t;
  return tp;
}

// Actor forward (networks.py:51-63) on [B][ldS] states.
// h1 is always materialised (input of layer 2); h2 only when h2 != nullptr.
// l1_done: h1 was already produced (first_layers_dev).
static void actor_fwd(ddpg_ctx* c, const float* base, const float* s, int B, float* h1,
                      float* h2, float* o, float* mu, bool l1_done = false) {
  const Layout& L = c->L;
  GemmEpi e = epi_none();
  Twin h1t;
  const TkPart tp = actor_l1_part(c, base, s, B, h1, &h1t);
  if (!l1_done && !thin_k_launch(c, "fwd", &tp, 1, B)) {
    e.out = h1t.p ? nullptr : h1;
    e.outh = h1t.p;
    e.h_plane_stride = h1t.ps;
    e.h_planes = c->hnp;
    e.ldo = c->ldAH1;
    e.bias = P(c, base, L.a[AB1]);
    e.act = 1;
    gemm_launch<L_RK, L_KR>(c, "fwd", s, c->ldS, P(c, base, L.a[AW1]), c->AH1, B, c->AH1, c->S,
                            e);
  }
  e = epi_none();
  e.out = h2;
  e.ldo = c->ldAH2;
  e.bias = P(c, base, L.a[AB2]);
  e.act = 1;
  e.proj = P(c, base, L.a[AW3]);
  e.proj_n = c->A;
  e.proj_sn = c->A;
  e.proj_sa = 1;
  e.proj_out = c->ppart;
  GemmPlan pl = gemm_launch<L_RK, L_KR>(c, "fwd_head", h1, c->ldAH1, P(c, base, L.a[AW2]),
                                        c->AH2, B, c->AH2, c->AH1, e);
  ProfScope ps(c, "actor_out", 0, 0);
  hipLaunchKernelGGL(actor_out_kernel, dim3(ceil_div(B * c->A, 256)), dim3(256), 0, c->cur,
                     c->ppart, pl.nt(c->AH2), B, c->A, c->cfg.action_scale, o, mu, c->ldA);
  HIP_TRY(hipGetLastError());
}

// Critic first layer + hidden layer (networks.py:147-161).  mode:
//   0: store h (train), proj(Wo) -> qpart
//   1: proj(Wo) -> qpart only (predict / target)
//   2: dh_pre = Wo[j] * elu'(h) -> dhp_out (action-gradient path, grad_ys = 1)
// Returns the number of qpart slabs (modes 0/1).
// The critic's first layer, [state branch | action branch] of the concat, as
// two thin-K parts.  The target path's concat is read only by the hidden
// layer: when that runs on the twin GEMM, only the twin is written.
static Twin critic_l1_parts(ddpg_ctx* c, const float* base, const float* s, const float* a, int B,
                            float* cat, TkPart tp[2]) {
  const Layout& L = c->L;
  int kh;
  const bool planes =
      (cat == c->tcat && gemm_h_ok<L_RK, L_KR>(c, cat, c->ldC, P(c, base, L.c[CWH]), c->CH2, B,
                                                c->CH2, 2 * c->CH1, 1, &kh)) ||
      (cat == c->cat && act_planes_only(c, ACT_CAT, B)) ||
      (cat == c->cat2 && act_planes_only(c, ACT_CAT2, B));
  const Twin ct = planes ? act_twin(c, cat) : Twin();
  tp[0] = tk_part(s, c->ldS, c->S, P(c, base, L.c[CWS]), c->CH1, 0, c->CH1, P(c, base, L.c[CBS]),
                  1, ct.p ? nullptr : cat, c->ldC);
  tp[1] = tk_part(a, c->ldA, c->A, P(c, base, L.c[CWA]), c->CH1, 0, c->CH1, P(c, base, L.c[CBA]),
                  1, ct.p ? nullptr : cat + c->CH1, c->ldC);
  if (ct.p)
    for (int i = 0; i < 2; ++i) {
      tp[i].outh = ct.p + i * c->CH1;
      tp[i].hps = ct.ps;
      tp[i].hnp = c->hnp;
    }
  return ct;
}

// l1_done: 0 compute both first-layer branches, 1 the state branch is
// already in `cat` (first_layers_dev), 2 both are.
static int critic_fwd(ddpg_ctx* c, const float* base, const float* s, const float* a, int B,
                      float* cat, float* h_out, int mode, float* dhp_out, int l1_done = 0) {
  const Layout& L = c->L;
  GemmEpi e = epi_none();
  int kh;
  TkPart tp[2];
  const Twin ct = critic_l1_parts(c, base, s, a, B, cat, tp);
  if (l1_done == 1) {
    if (!thin_k_launch(c, "fwd", &tp[1], 1, B)) {
      e.ldo = c->ldC;
      e.act = 1;
      e.h_plane_stride = ct.ps;
      e.h_planes = c->hnp;
      e.out = ct.p ? nullptr : cat + c->CH1;
      e.outh = ct.p ? ct.p + c->CH1 : nullptr;
      e.bias = P(c, base, L.c[CBA]);
      gemm_launch<L_RK, L_KR>(c, "fwd", a, c->ldA, P(c, base, L.c[CWA]), c->CH1, B, c->CH1,
                              c->A, e);
    }
  } else if (l1_done == 0 && !thin_k_launch(c, "fwd", tp, 2, B)) {  // each branch on its own
    e.ldo = c->ldC;
    e.act = 1;
    e.h_plane_stride = ct.ps;
    e.h_planes = c->hnp;
    if (!thin_k_launch(c, "fwd", &tp[0], 1, B)) {
      e.out = ct.p ? nullptr : cat;
      e.outh = ct.p;
      e.bias = P(c, base, L.c[CBS]);
      gemm_launch<L_RK, L_KR>(c, "fwd", s, c->ldS, P(c, base, L.c[CWS]), c->CH1, B, c->CH1,
                              c->S, e);
    }
    if (!thin_k_launch(c, "fwd", &tp[1], 1, B)) {
      e.out = ct.p ? nullptr : cat + c->CH1;
      e.outh = ct.p ? ct.p + c->CH1 : nullptr;
      e.bias = P(c, base, L.c[CBA]);
      gemm_launch<L_RK, L_KR>(c, "fwd", a, c->ldA, P(c, base, L.c[CWA]), c->CH1, B, c->CH1,
                              c->A, e);
    }
  }
  e = epi_none();
  e.bias = P(c, base, L.c[CBH]);
  e.act = 1;
  if (mode == 2) {
    e.post = 2;
    e.pw = P(c, base, L.c[CWO]);
    e.out = dhp_out;
    e.ldo = c->ldCH2;
    // dh_pre of the action-gradient path feeds only the dx_da GEMM
    const float* whA = P(c, base, L.c[CWH]) + (size_t)c->CH1 * c->CH2;
    if (gemm_h_ok<L_RK, L_RK>(c, dhp_out, c->ldCH2, whA, c->CH2, B, c->CH1, c->CH2, 1, &kh)) {
      const Twin dt = act_twin(c, dhp_out);
      e.out = nullptr;
      e.outh = dt.p;
      e.h_plane_stride = dt.ps;
      e.h_planes = c->hnp;
    }
  } else {
    e.out = (mode == 0) ? h_out : nullptr;
    e.ldo = c->ldCH2;
    e.proj = P(c, base, L.c[CWO]);
    e.proj_n = 1;
    e.proj_sn = 1;
    e.proj_sa = 0;
    e.proj_out = c->qpart;
  }
  GemmPlan pl = gemm_launch<L_RK, L_KR>(c, mode == 2 ? "fwd_dhead" : "fwd_head", cat, c->ldC,
                                        P(c, base, L.c[CWH]), c->CH2, B, c->CH2, 2 * c->CH1, e);
  return pl.nt(c->CH2);
}

// dQ/da of the (already updated) online critic at (s, a): networks.py:143.
// Writes da (optional, [B][ldA]) and dz3 = actor grad_ys chain (optional).
static void critic_action_grad(ddpg_ctx* c, const float* s, const float* a, int B, float* da,
                               float* dz3, const float* o) {
  const Layout& L = c->L;
  critic_fwd(c, c->theta, s, a, B, c->cat2, nullptr, 2, c->dhp2);
  GemmEpi e = epi_none();
  e.post = 1;
  epi_aux(c, e, ACT_CAT2, B, c->cat2 + c->CH1, c->ldC);
  e.proj = P(c, c->theta, L.c[CWA]);
  e.proj_n = c->A;
  e.proj_sn = 1;
  e.proj_sa = c->CH1;
  e.proj_out = c->ppart;
  // B operand = Wh[CH1:2CH1, :]^T  (NK: element (k=j, n=i) at Wh[(CH1+i)*CH2 + j])
  GemmPlan pl = gemm_launch<L_RK, L_RK>(c, "dx_da", c->dhp2, c->ldCH2,
                                        P(c, c->theta, L.c[CWH]) + (size_t)c->CH1 * c->CH2,
                                        c->CH2, B, c->CH1, c->CH2, e);
  ProfScope ps(c, "action_grad", 0, 0);
  hipLaunchKernelGGL(action_grad_kernel, dim3(ceil_div(B * c->A, 256)), dim3(256), 0, c->cur,
                     c->ppart, pl.nt(c->CH1), B, c->A, B, o, c->ldA, c->cfg.action_scale, da,
                     dz3);
  HIP_TRY(hipGetLastError());
}

// Weight gradient dW[M][N] = A^T . B over K = B rows (A [K][lda] M columns,
// B [K][ldb] N columns; split-K slabs [split][M][N] or `direct`): on the
// skinny kernel (skinny.h) when one side is at most 64 wide and the other a
// multiple of 4 (>= 128), with the narrow operand's row holding every column
// its NG-wide tiles read; otherwise on the GEMMs.
static GemmPlan wgrad_launch(ddpg_ctx* c, const float* A, int lda, const float* B, int ldb, int M,
                             int N, int K, float* slab, int cap, float* direct) {
  const bool a_narrow = M <= SK_NMAX && N >= 128;
  const bool b_narrow = N <= SK_NMAX && M >= 128 && !a_narrow;
  const float* nar = a_narrow ? A : B;
  const int ldn = a_narrow ? lda : ldb, nn = a_narrow ? M : N;
  const int ldw = a_narrow ? ldb : lda, nw = a_narrow ? N : M;
  // 16 narrow columns per wave above 16 (one 128 KB reduction: 1 block per
  // CU, 256 blocks); 8 at or below (64 KB, 2 blocks per CU, 512 blocks) --
  // measured, profiles/r3/skinny_variants.txt
  const int ng = (nn > 16 && rup(nn, 16) <= ldn) ? 16 : 8;
  const int ntn = ceil_div(std::max(nn, 1), ng);
  if (c->sw.skinny && (a_narrow || b_narrow) && nw % 4 == 0 && ldw % 4 == 0 &&
      ntn * ng <= ldn && aligned16(a_narrow ? B : A)) {
    GemmPlan p;
    const int ntw = ceil_div(nw, SK_WT), tiles = ntw * ntn;
    int splits = std::min(cap, std::max(1, (ng == 8 ? 512 : 256) / tiles));
    int kc = rup(ceil_div(K, splits), SK_WAVES);
    splits = ceil_div(K, kc);
    p.splits = splits;
    SkArgs a;
    a.N = nar;
    a.ldn = ldn;
    a.nn = nn;
    a.W = a_narrow ? B : A;
    a.ldw = ldw;
    a.nw = nw;
    a.B = K;
    a.kc = kc;
    a.ntw = ntw;
    a.ntn = ntn;
    a.narrow_rows = a_narrow ? 1 : 0;
    if (splits == 1 && direct) {
      a.out = direct;
      a.split_stride = 0;
      p.direct = true;
    } else {
      a.out = slab;
      a.split_stride = (long long)M * N;
    }
    ProfScope ps(c, "skinny_wgrad_kernel|wgrad", 2.0 * M * N * (double)K,
                 4.0 * ((double)K * (M + N) + (double)M * N * splits));
    if (ng == 8)
      hipLaunchKernelGGL(skinny_wgrad_kernel<8>, dim3(tiles * splits), dim3(SK_NT),
                         sk_lds_bytes(8), c->cur, a);
    else
      hipLaunchKernelGGL(skinny_wgrad_kernel<16>, dim3(tiles * splits), dim3(SK_NT),
                         sk_lds_bytes(16), c->cur, a);
    HIP_TRY(hipGetLastError());
    return p;
  }
  GemmEpi e = epi_none();
  e.out = slab;
  e.ldo = N;
  e.out_split_stride = (long long)M * N;
  return gemm_launch<L_KR, L_KR>(c, "wgrad", A, lda, B, ldb, M, N, K, e, 0, cap, direct);
}

static void add_seg(ReduceTable& t, const float* src, float* dst, long long stride, int nslab,
                    long long count) {
  ReduceSeg& s = t.seg[t.nseg++];
  s.src = src;
  s.dst = dst;
  s.slab_stride = stride;
  s.nslab = nslab;
  s.count = count;
  s.vec4 = (count % 4 == 0) && (stride % 4 == 0) && aligned16(src) && aligned16(dst);
}

// a weight-gradient GEMM's slabs, unless it wrote the gradient directly
static void add_wgrad(ReduceTable& t, const GemmPlan& p, const float* slab, float* dst,
                      long long count) {
  if (!p.direct) add_seg(t, slab, dst, count, p.splits, count);
}

static void reduce_launch(ddpg_ctx* c, const char* name, ReduceTable& tab) {
  long long maxc = 1;
  double bytes = 0;
  for (int i = 0; i < tab.nseg; ++i) {
    maxc = std::max(maxc, tab.seg[i].count);
    bytes += (double)tab.seg[i].count * 4.0 * (tab.seg[i].nslab + 1);
  }
  ProfScope ps(c, name, 0, bytes);
  const int bx = (int)std::min<long long>(1024, std::max<long long>(1, (maxc / 4 + 63) / 64));
  hipLaunchKernelGGL(reduce_slabs_kernel, dim3(bx, tab.nseg), dim3(256), 0, c->cur, tab);
  HIP_TRY(hipGetLastError());
}

static void nccl_try(ncclResult_t r) {
  if (r != ncclSuccess) throw DdpgError(DDPG_ECOMM, ncclGetErrorString(r));
}

// `to` waits for the work queued so far on `from` (comm-stream events cev)
static void cs_link(ddpg_ctx* c, int ev, hipStream_t from, hipStream_t to) {
  if (from == to) return;
  HIP_TRY(hipEventRecord(c->cev[ev], from));
  HIP_TRY(hipStreamWaitEvent(to, c->cev[ev], 0));
}

// In-place RCCL sums of up to 2 disjoint ranges of the flat grad buffer, on
// the comm stream after the work queued so far on c->cur (one group: one
// launch).  The caller joins cs back before the gradients are read.
// with_stats: the all-gather of the step's {q_max, loss} joins the same group
// (one collective launch, one latency on the critical path instead of two);
// stats_allreduce_on_cs then only reduces the gathered values.
// window (profiling only): open an exchange-overlap record on the producing
// stream, closed by the next join_cs -- the compute that stream runs between
// issuing this exchange and waiting for it (bench.py's projected scaling).
static void allreduce_on_cs(ddpg_ctx* c, int ev, const char* name, float* b0, size_t n0,
                            float* b1 = nullptr, size_t n1 = 0, bool with_stats = false,
                            const char* window = nullptr) {
  if (!c->comm) return;
  cs_link(c, ev, c->cur, c->cs);
  const hipStream_t prev = c->cur;
  if (window && c->prof && c->win_rec < 0) {
    ProfRec rec{window, ev_get(c), ev_get(c), 0.0, (double)n0 * 4.0};
    HIP_TRY(hipEventRecord(rec.e0, prev));
    c->prof_recs.push_back(rec);
    c->win_rec = (int)c->prof_recs.size() - 1;
  }
  c->cur = c->cs;
  if (c->test_cs_spin) {
    // test hook: the exchanged ranges doubled after a delay, on cs ahead of
    // the group -- a consumer not ordered behind cs reads them undoubled
    hipLaunchKernelGGL(cs_spin_scale_kernel, dim3(256), dim3(256), 0, c->cs, b0, (long long)n0,
                       b1, (long long)n1, c->test_cs_spin);
    HIP_TRY(hipGetLastError());
  }
  {
    ProfScope ps(c, name, 0, (double)(n0 + n1) * 4.0 + (with_stats ? 8.0 * c->cworld : 0.0));
    nccl_try(ncclGroupStart());
    if (n0) nccl_try(ncclAllReduce(b0, b0, n0, ncclFloat, ncclSum, c->comm, c->cs));
    if (n1) nccl_try(ncclAllReduce(b1, b1, n1, ncclFloat, ncclSum, c->comm, c->cs));
    if (with_stats)
      nccl_try(ncclAllGather(c->dstats, c->dstats_all, 2, ncclFloat, c->comm, c->cs));
    nccl_try(ncclGroupEnd());
  }
  c->cur = prev;
}

// the logged stats of a data-parallel step are the
// global-batch ones (ddpg.py:102-103) -- max over ranks of max(Q) and the sum
// of the ranks' loss shares (each already scaled by 1/B_global).  One
// all-gather of every rank's {q_max, loss}, then an ordered reduction that
// every rank computes identically; it also feeds the running sums.  On the
// comm stream, after the critic all-reduce.
static void stats_allreduce_on_cs(ddpg_ctx* c, bool gathered = false) {
  if (!c->comm) return;
  const hipStream_t prev = c->cur;
  c->cur = c->cs;
  {
    ProfScope ps(c, "rccl_stats", 0, gathered ? 0.0 : 8.0 * c->cworld);
    if (!gathered)
      nccl_try(ncclAllGather(c->dstats, c->dstats_all, 2, ncclFloat, c->comm, c->cs));
    hipLaunchKernelGGL(stats_reduce_kernel, dim3(1), dim3(64), 0, c->cs, c->dstats_all, c->cworld,
                       c->dstats, c->dacc);
    HIP_TRY(hipGetLastError());
  }
  c->cur = prev;
}

// the consumer stream (c->cur) waits for every collective queued on cs
static void join_cs(ddpg_ctx* c, int ev) {
  if (!c->comm) return;
  if (c->win_rec >= 0) {  // close the exchange-overlap window on the consumer stream
    HIP_TRY(hipEventRecord(c->prof_recs[c->win_rec].e1, c->cur));
    c->win_rec = -1;
  }
  cs_link(c, ev, c->cs, c->cur);
}

// TF ApplyAdam over one network's flat region.  advance: also advance its
// beta powers right after (1:1 API path).  soft (fused step): the same pass
// also soft-updates this network's targets from the new parameters; the
// fused step then advances both networks' beta powers at its end.
static void adam_launch(ddpg_ctx* c, int net, bool advance, bool soft = false) {
  const size_t b = net == 0 ? c->L.actor_begin : c->L.critic_begin;
  const size_t e = net == 0 ? c->L.actor_end : c->L.critic_end;
  const long long n = (long long)(e - b);
  const float lr = net == 0 ? c->cfg.actor_lr : c->cfg.critic_lr;
  int blocks = (int)std::min<long long>(4096, std::max<long long>(1, (n / 4 + 255) / 256));
  c->sb_shadow_ok = false;
  {
    const float tau = c->cfg.tau, omt = (float)(1.0 - (double)tau);
    ProfScope ps(c, soft ? "adam+soft_update" : "adam", 0, (soft ? 40.0 : 28.0) * n);
    // keeps theta's (and theta''s) twin current, or leaves it stale if it already was
    __bf16* tw = (c->hnp && c->wtw_ok) ? c->wtw + b : nullptr;
    __bf16* ttw = (c->hnp && c->wtw_ok) ? c->wtw + (size_t)c->hnp * c->L.total + b : nullptr;
    hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, c->cur, c->theta + b,
                       c->adam_m + b, c->adam_v + b, c->grad + b, n, c->dpw + 2 * net, lr,
                       c->cfg.beta1, c->cfg.beta2, c->cfg.epsilon, tw, (long long)c->L.total,
                       c->hnp, soft ? c->target + b : nullptr, tau, omt, soft ? ttw : nullptr);
    HIP_TRY(hipGetLastError());
  }
  if (advance) {
    hipLaunchKernelGGL(advance_powers_kernel, dim3(1), dim3(1), 0, c->cur, c->dpw, 1 << net,
                       c->cfg.beta1, c->cfg.beta2);
    HIP_TRY(hipGetLastError());
  }
}

// Fork/join between the ctx streams (par == false keeps everything on cur).
static void fork_to(ddpg_ctx* c, int ev, hipStream_t from, hipStream_t to) {
  if (from == to) return;
  HIP_TRY(hipEventRecord(c->fj[ev], from));
  HIP_TRY(hipStreamWaitEvent(to, c->fj[ev], 0));
}

// Critic update on rows already in c->s / c->a with targets in c->y.
// networks.py:130-137,170-175 (+ RCCL sum over ranks for world > 1).
// nq < 0: run the critic forward here; otherwise it already ran (fused step,
// concurrently with the target path) and left nq Wo-projection slabs.
// par: run dWh concurrently with dcat on aux[0].
static void critic_train_dev(ddpg_ctx* c, int B, float inv_b, bool fused, int nq = -1,
                             bool par = false) {
  const Layout& L = c->L;
  if (nq < 0) nq = critic_fwd(c, c->theta, c->s, c->a, B, c->cat, c->h, 0, nullptr);
  {
    ProfScope ps(c, "critic_loss", 0, 0);
    // world > 1: the per-step stats are reduced over ranks below, then accumulated
    // fused step: the TD target of ddpg.py:90-100 formed here (td_nqt)
    TdTarget td;
    memset(&td, 0, sizeof td);
    if (fused && c->td_nqt > 0) {
      td.qpart = c->qpart_t;
      td.NT = c->td_nqt;
      td.bo = P(c, c->target, L.c[CBO]);
      td.r = c->r;
      td.t = c->t;
      td.gamma = c->cfg.gamma;
    }
    c->td_nqt = 0;
    hipLaunchKernelGGL(critic_loss_kernel, dim3(ceil_div(B, 256)), dim3(256), 0, c->cur,
                       c->qpart, nq, B, P(c, c->theta, L.c[CBO]), c->y, inv_b, c->q, c->dq,
                       c->lpart, td);
    HIP_TRY(hipGetLastError());
  }
  // column quads when the widths allow; dh_pre's twin is written here
  const bool hq = c->CH2 % 4 == 0 && c->ldCH2 % 4 == 0;
  const int hrows = hq ? kHeadRows4 : kHeadRows;
  const int nchunk = ceil_div(B, hrows);
  float* part_dWo = c->headpart;
  float* part_dbh = c->headpart + (size_t)nchunk * c->CH2;
  float* part_dbo = part_dbh + (size_t)nchunk * c->CH2;
  // dh_pre feeds dWh and dcat only: when both run on the twin GEMM, only its
  // twin is written
  int kh;
  const bool dhp_twin_only =
      gemm_h_ok<L_KR, L_KR>(c, c->cat, c->ldC, c->dhp, c->ldCH2, 2 * c->CH1, c->CH2, B, 0, &kh) &&
      gemm_h_ok<L_RK, L_RK>(c, c->dhp, c->ldCH2, P(c, c->theta, L.c[CWH]), c->CH2, B,
                            2 * c->CH1, c->CH2, 1, &kh);
  {
    ProfScope ps(c, "critic_head_bwd", 0, (double)B * c->CH2 * 8.0);
    if (hq) {
      const Twin tw = act_twin(c, c->dhp);
      hipLaunchKernelGGL(critic_head_bwd4_kernel, dim3(ceil_div(c->CH2 / 4, 64), nchunk),
                         dim3(256), 0, c->cur, c->h, c->ldCH2, c->dq, P(c, c->theta, L.c[CWO]),
                         B, c->CH2, hrows, dhp_twin_only ? nullptr : c->dhp, c->ldCH2, part_dWo,
                         part_dbh, part_dbo, tw.p,
                         tw.ps, c->hnp, c->lpart, ceil_div(B, 256), inv_b, c->dstats,
                         c->comm ? nullptr : c->dacc);
    } else {
      if (act_twin(c, c->dhp).p) throw einval("dh_pre twin needs CH2 %% 4 == 0");
      hipLaunchKernelGGL(critic_head_bwd_kernel, dim3(ceil_div(c->CH2, 256), nchunk), dim3(256), 0,
                         c->cur, c->h, c->ldCH2, c->dq, P(c, c->theta, L.c[CWO]), B, c->CH2,
                         hrows, c->dhp, c->ldCH2, part_dWo, part_dbh, part_dbo, c->lpart,
                         ceil_div(B, 256), inv_b, c->dstats, c->comm ? nullptr : c->dacc);
    }
    HIP_TRY(hipGetLastError());
  }
  // dWh = cat^T . dh_pre   (split-K slabs; on aux[0] when par)
  const hipStream_t main = c->cur;
  if (par) {
    fork_to(c, 4, main, c->aux[0]);
    c->cur = c->aux[0];
  }
  GemmEpi e = epi_none();
  e.out = c->slab_Wh;
  e.ldo = c->CH2;
  e.out_split_stride = (long long)2 * c->CH1 * c->CH2;
  GemmPlan pWh = gemm_launch<L_KR, L_KR>(c, "wgrad", c->cat, c->ldC, c->dhp, c->ldCH2, 2 * c->CH1,
                                         c->CH2, B, e, 0, c->split_cap_Wh,
                                         c->grad + L.c[CWH].off);
  float* G = c->grad;
  const long long nWh = (long long)2 * c->CH1 * c->CH2;
  if (c->comm) {
    // data parallel: dWh (96 % of the critic's gradient bytes) is reduced and
    // its all-reduce started now, under the dcat / dWs / dWa GEMMs below
    ReduceTable t1;
    t1.nseg = 0;
    add_wgrad(t1, pWh, c->slab_Wh, G + L.c[CWH].off, nWh);
    if (t1.nseg) reduce_launch(c, "grad_reduce", t1);
    allreduce_on_cs(c, 0, "rccl_allreduce", G + L.c[CWH].off, (size_t)nWh, nullptr, 0, false,
                    "xwin|critic");
  }
  c->cur = main;
  // dcat = dh_pre . Wh^T * elu'(cat);  column sums -> [dbs | dba]
  e = epi_none();
  e.post = 1;
  epi_aux(c, e, ACT_CAT, B, c->cat, c->ldC);
  e.out = c->dcat;
  e.ldo = c->ldC;
  e.colsum = c->colpart;
  e.ld_colsum = 2 * c->CH1;
  GemmPlan pdc = gemm_launch<L_RK, L_RK>(c, "dx", c->dhp, c->ldCH2, P(c, c->theta, L.c[CWH]),
                                         c->CH2, B, 2 * c->CH1, c->CH2, e);
  const int mt = pdc.mt(B);
  // dWs = s^T . dcs ; dWa = a^T . dca
  GemmPlan pWs = wgrad_launch(c, c->s, c->ldS, c->dcat, c->ldC, c->S, c->CH1, B, c->slab_Ws,
                              c->split_cap_Ws, c->grad + L.c[CWS].off);
  GemmPlan pWa = wgrad_launch(c, c->a, c->ldA, c->dcat + c->CH1, c->ldC, c->A, c->CH1, B,
                              c->slab_Wa, c->split_cap_Wa, c->grad + L.c[CWA].off);
  if (par) fork_to(c, 5, c->aux[0], main);  // join dWh
  // gather every critic gradient into the flat grad buffer
  ReduceTable tab;
  tab.nseg = 0;
  add_wgrad(tab, pWs, c->slab_Ws, G + L.c[CWS].off, (long long)c->S * c->CH1);
  add_seg(tab, c->colpart, G + L.c[CBS].off, 2 * c->CH1, mt, c->CH1);
  add_wgrad(tab, pWa, c->slab_Wa, G + L.c[CWA].off, (long long)c->A * c->CH1);
  add_seg(tab, c->colpart + c->CH1, G + L.c[CBA].off, 2 * c->CH1, mt, c->CH1);
  if (!c->comm) add_wgrad(tab, pWh, c->slab_Wh, G + L.c[CWH].off, nWh);
  add_seg(tab, part_dbh, G + L.c[CBH].off, c->CH2, nchunk, c->CH2);
  add_seg(tab, part_dWo, G + L.c[CWO].off, c->CH2, nchunk, c->CH2);
  add_seg(tab, part_dbo, G + L.c[CBO].off, 1, nchunk, 1);
  reduce_launch(c, "grad_reduce", tab);
  if (c->comm) {
    // the rest of the critic ([Ws bs Wa ba] and [bh Wo bo]) behind dWh on the
    // comm stream, then the stats; Adam waits for all of it
    allreduce_on_cs(c, 1, "rccl_allreduce", G + L.critic_begin, L.c[CWH].off - L.critic_begin,
                    G + L.c[CBH].off, L.critic_end - L.c[CBH].off, true);
    stats_allreduce_on_cs(c, true);
    join_cs(c, 2);
  }
  adam_launch(c, 1, !fused, fused);
}

// Actor update given dz3 (= TanhGrad chain of -dQ/da) and the forward
// activations h1, h2 of c->s.  networks.py:39-47,71-75.
// par: weight-gradient GEMMs (dW3, dW2) run on aux[0] beside the dX chain.
static void actor_train_dev(ddpg_ctx* c, int B, bool fused, bool par = false) {
  const Layout& L = c->L;
  float* G = c->grad;
  const hipStream_t main = c->cur;
  // dW3 = h2^T . dz3
  if (par) {
    fork_to(c, 6, main, c->aux[0]);
    c->cur = c->aux[0];
  }
  GemmPlan pW3 = wgrad_launch(c, c->h2, c->ldAH2, c->dz3, c->ldA, c->AH2, c->A, B, c->slab_W3,
                              c->split_cap_W3, G + L.a[AW3].off);
  GemmEpi e = epi_none();
  c->cur = main;
  // dz2 = (dz3 . W3^T) * elu'(h2); colsum -> db2
  // dz2 feeds dW2 and dz1 only; dz1 feeds dW1 only: twin-only when those run
  // on the twin GEMM
  int kh;
  const Twin dz2t =
      (gemm_h_ok<L_KR, L_KR>(c, c->h1, c->ldAH1, c->dz2, c->ldAH2, c->AH1, c->AH2, B, 0, &kh) &&
       gemm_h_ok<L_RK, L_RK>(c, c->dz2, c->ldAH2, P(c, c->theta, L.a[AW2]), c->AH2, B, c->AH1,
                             c->AH2, 1, &kh))
          ? act_twin(c, c->dz2)
          : Twin();
  const Twin dz1t =
      gemm_h_ok<L_KR, L_KR>(c, c->s, c->ldS, c->dz1, c->ldAH1, c->S, c->AH1, B, 0, &kh)
          ? act_twin(c, c->dz1)
          : Twin();
  TkPart tp = tk_part(c->dz3, c->ldA, c->A, P(c, c->theta, L.a[AW3]), c->A, 1, c->AH2, nullptr,
                      0, dz2t.p ? nullptr : c->dz2, c->ldAH2);
  tp.outh = dz2t.p;
  tp.hps = dz2t.ps;
  tp.hnp = c->hnp;
  tp.aux = c->h2;
  tp.ldaux = c->ldAH2;
  tp.colsum = c->colpart;
  tp.ld_colsum = c->AH2;
  int mt2 = thin_k_launch(c, "dx", &tp, 1, B);
  if (!mt2) {
    e = epi_none();
    e.post = 1;
    e.aux = c->h2;
    e.ldaux = c->ldAH2;
    e.out = dz2t.p ? nullptr : c->dz2;
    e.outh = dz2t.p;
    e.h_plane_stride = dz2t.ps;
    e.h_planes = c->hnp;
    e.ldo = c->ldAH2;
    e.colsum = c->colpart;
    e.ld_colsum = c->AH2;
    GemmPlan pz2 = gemm_launch<L_RK, L_RK>(c, "dx", c->dz3, c->ldA, P(c, c->theta, L.a[AW3]),
                                           c->A, B, c->AH2, c->A, e);
    mt2 = pz2.mt(B);
  }
  // dW2 = h1^T . dz2   (aux[0] waits for dz2, then runs beside dz1)
  if (par) {
    fork_to(c, 7, main, c->aux[0]);
    c->cur = c->aux[0];
  }
  e = epi_none();
  e.out = c->slab_W2;
  e.ldo = c->AH2;
  e.out_split_stride = (long long)c->AH1 * c->AH2;
  GemmPlan pW2 = gemm_launch<L_KR, L_KR>(c, "wgrad", c->h1, c->ldAH1, c->dz2, c->ldAH2, c->AH1,
                                         c->AH2, B, e, 0, c->split_cap_W2, G + L.a[AW2].off);
  const long long nW2 = (long long)c->AH1 * c->AH2;
  if (c->comm) {
    // data parallel: dW2 (the bulk of the actor's gradient) reduced and its
    // all-reduce started now, under the dz1 / dW1 GEMMs
    ReduceTable t1;
    t1.nseg = 0;
    add_wgrad(t1, pW2, c->slab_W2, G + L.a[AW2].off, nW2);
    if (t1.nseg) reduce_launch(c, "grad_reduce", t1);
    allreduce_on_cs(c, 3, "rccl_allreduce", G + L.a[AW2].off, (size_t)nW2, nullptr, 0, false,
                    "xwin|actor");
  }
  c->cur = main;
  // dz1 = (dz2 . W2^T) * elu'(h1); colsum -> db1
  float* colpart1 = c->colpart + (size_t)mt2 * c->AH2;
  e = epi_none();
  e.post = 1;
  epi_aux(c, e, ACT_H1, B, c->h1, c->ldAH1);
  e.out = dz1t.p ? nullptr : c->dz1;
  e.outh = dz1t.p;
  e.h_plane_stride = dz1t.ps;
  e.h_planes = c->hnp;
  e.ldo = c->ldAH1;
  e.colsum = colpart1;
  e.ld_colsum = c->AH1;
  GemmPlan pz1 = gemm_launch<L_RK, L_RK>(c, "dx", c->dz2, c->ldAH2, P(c, c->theta, L.a[AW2]),
                                         c->AH2, B, c->AH1, c->AH2, e);
  // dW1 = s^T . dz1
  GemmPlan pW1 = wgrad_launch(c, c->s, c->ldS, c->dz1, c->ldAH1, c->S, c->AH1, B, c->slab_W1,
                              c->split_cap_W1, G + L.a[AW1].off);
  if (par) fork_to(c, 3, c->aux[0], main);  // join dW3, dW2
  ReduceTable tab;
  tab.nseg = 0;
  add_wgrad(tab, pW1, c->slab_W1, G + L.a[AW1].off, (long long)c->S * c->AH1);
  add_seg(tab, colpart1, G + L.a[AB1].off, c->AH1, pz1.mt(B), c->AH1);
  if (!c->comm) add_wgrad(tab, pW2, c->slab_W2, G + L.a[AW2].off, nW2);
  add_seg(tab, c->colpart, G + L.a[AB2].off, c->AH2, mt2, c->AH2);
  add_wgrad(tab, pW3, c->slab_W3, G + L.a[AW3].off, (long long)c->AH2 * c->A);
  reduce_launch(c, "grad_reduce", tab);
  if (c->comm) {  // [W1 b1] and [b2 W3] behind dW2 on the comm stream
    allreduce_on_cs(c, 4, "rccl_allreduce", G + L.actor_begin, L.a[AW2].off - L.actor_begin,
                    G + L.a[AB2].off, L.actor_end - L.a[AB2].off);
    join_cs(c, 5);
  }
  adam_launch(c, 0, !fused, fused);
}

// Soft target update (networks.py:34-37) over the selected networks; pw_mask
// additionally advances those networks' Adam beta powers (fused step).
static void soft_update_dev(ddpg_ctx* c, int mask, int pw_mask) {
  const float tau = c->cfg.tau;
  const float omt = (float)(1.0 - (double)tau);
  size_t b, e;
  if ((mask & DDPG_SOFT_ACTOR) && (mask & DDPG_SOFT_CRITIC)) {
    b = c->L.actor_begin;
    e = c->L.critic_end;
  } else if (mask & DDPG_SOFT_ACTOR) {
    b = c->L.actor_begin;
    e = c->L.actor_end;
  } else if (mask & DDPG_SOFT_CRITIC) {
    b = c->L.critic_begin;
    e = c->L.critic_end;
  } else {
    return;
  }
  const long long n = (long long)(e - b);
  int blocks = (int)std::min<long long>(4096, std::max<long long>(1, (n / 4 + 255) / 256));
  ProfScope ps(c, "soft_update", 0, 12.0 * n);
  __bf16* tw = (c->hnp && c->wtw_ok) ? c->wtw + (size_t)c->hnp * c->L.total + b : nullptr;
  hipLaunchKernelGGL(soft_update_kernel, dim3(blocks), dim3(256), 0, c->cur, c->theta + b,
                     c->target + b, n, tau, omt, c->dpw, pw_mask, c->cfg.beta1, c->cfg.beta2,
                     tw, (long long)c->L.total, c->hnp);
  HIP_TRY(hipGetLastError());
}

// One full learner step (ddpg.py:86-113) on rows already gathered into
// c->s, c->a, c->r, c->t, c->s2 (B local rows, inv_b = 1/B_global).
// Dependency-preserving concurrency (same results, bitwise): the target path
// (aux[0]), the online actor forward (aux[1]) and the online critic forward
// (main) are independent until the critic loss; inside the backward passes
// the weight-gradient GEMMs run beside the dX chain.
// The five first layers of a large-batch step that depend only on the batch
// and the pre-step parameters (target actor on s2, the target critic's state
// branch on s2, actor on s, the critic's state and action branches on (s, a))
// as ONE thin-K launch: one ramp and tail instead of four, 5 x 512 blocks to
// fill the chip.  Returns false (nothing launched) when a part is not
// thin-K-eligible; the per-network paths then compute them as before.
static bool first_layers_dev(ddpg_ctx* c, int B) {
  if (!c->sw.thin_k || !c->sw.l1_batch) return false;
  TkPart tp[TK_MAXP], tc[2];
  tp[0] = actor_l1_part(c, c->target, c->s2, B, c->th1, nullptr);
  critic_l1_parts(c, c->target, c->s2, c->ta2, B, c->tcat, tc);
  tp[1] = tc[0];
  tp[2] = actor_l1_part(c, c->theta, c->s, B, c->h1, nullptr);
  critic_l1_parts(c, c->theta, c->s, c->a, B, c->cat, tc);
  tp[3] = tc[0];
  tp[4] = tc[1];
  return thin_k_launch(c, "fwd_l1", tp, TK_MAXP, B) != 0;
}

static void learner_step_dev(ddpg_ctx* c, int B, float inv_b) {
  const hipStream_t s0 = c->cur;
  const hipStream_t s1 = c->par ? c->aux[0] : s0, s2 = c->par ? c->aux[1] : s0;
  // ddpg.py:90-109's batch-only first layers, all at once (every later use
  // reads them with the same pre-step parameters)
  const bool l1 = first_layers_dev(c, B);
  fork_to(c, 0, s0, s1);
  fork_to(c, 0, s0, s2);
  // target_q = critic.predict_target(s2, actor.predict_target(s2))  ddpg.py:90
  c->cur = s1;
  std::swap(c->ppart, c->ppart_t);
  std::swap(c->qpart, c->qpart_t);
  actor_fwd(c, c->target, c->s2, B, c->th1, nullptr, nullptr, c->ta2, l1);
  const int nqt =
      critic_fwd(c, c->target, c->s2, c->ta2, B, c->tcat, nullptr, 1, nullptr, l1 ? 1 : 0);
  std::swap(c->ppart, c->ppart_t);
  std::swap(c->qpart, c->qpart_t);
  // y = r + gamma (1 - t) Q'(s2, mu') is formed by the critic loss kernel from
  // the target partials now in qpart_t (critic_train_dev, td_nqt)
  c->td_nqt = nqt;
  // a_outs = actor.predict(s)  ddpg.py:106 (actor params are unchanged until actor.train)
  c->cur = s2;
  actor_fwd(c, c->theta, c->s, B, c->h1, c->h2, c->o, c->mu, l1);
  // critic.train(s, a, y)  ddpg.py:100: forward now, loss once y is ready
  c->cur = s0;
  const int nq = critic_fwd(c, c->theta, c->s, c->a, B, c->cat, c->h, 0, nullptr, l1 ? 2 : 0);
  fork_to(c, 1, s1, s0);  // join target path (y)
  critic_train_dev(c, B, inv_b, true, nq, c->par);
  // grads = critic.action_gradients(s, a_outs)  ddpg.py:107 (updated critic)
  fork_to(c, 2, s2, s0);  // join online actor forward (h1, h2, o, mu)
  critic_action_grad(c, c->s, c->mu, B, nullptr, c->dz3, c->o);
  // actor.train(s, grads[0])  ddpg.py:109  (forward above reused: same params)
  actor_train_dev(c, B, true, c->par);
  // actor/critic.update_target_network()  ddpg.py:112-113: done inside each
  // network's Adam pass above; here both Adam power updates (_finish)
  hipLaunchKernelGGL(advance_powers_kernel, dim3(1), dim3(1), 0, c->cur, c->dpw, 3,
                     c->cfg.beta1, c->cfg.beta2);
  HIP_TRY(hipGetLastError());
}

// Rebuild the W^T shadows of the small path after a parameter write outside
// it.  Eager (never captured into a step graph): the graph itself keeps the
// shadows current through sb_wgrad_adam.
static void sb_refresh_shadows(ddpg_ctx* c) {
  if (!c->sb_ok || c->sb_shadow_ok) return;
  const Layout& L = c->L;
  hipLaunchKernelGGL(sb_transpose_kernel, dim3(64), dim3(256), 0, c->stream,
                     c->theta + L.c[CWH].off, 2 * c->CH1, c->CH2, c->sb_whT);
  hipLaunchKernelGGL(sb_transpose_kernel, dim3(64), dim3(256), 0, c->stream,
                     c->theta + L.a[AW2].off, c->AH1, c->AH2, c->sb_w2T);
  HIP_TRY(hipGetLastError());
  c->sb_shadow_ok = true;
}

// Arguments of the small-batch kernels (rb may be null: action selection).
static SbArgs sb_args(ddpg_ctx* c, ddpg_replay* rb, int B, float inv_b) {
  const Layout& L = c->L;
  SbArgs a;
  memset(&a, 0, sizeof a);
  a.B = B;
  a.S = c->S;
  a.A = c->A;
  a.AH1 = c->AH1;
  a.AH2 = c->AH2;
  a.CH1 = c->CH1;
  a.CH2 = c->CH2;
  a.LX = rup(std::max(c->S, c->A), 4);
  a.LW = rup(std::max(std::max(c->AH1, c->AH2), std::max(2 * c->CH1, c->CH2)), 4);
  a.inv_b = inv_b;
  a.gamma = c->cfg.gamma;
  a.scale = c->cfg.action_scale;
  a.tau = c->cfg.tau;
  a.omt = (float)(1.0 - (double)c->cfg.tau);
  a.b1 = c->cfg.beta1;
  a.b2 = c->cfg.beta2;
  a.lr_a = c->cfg.actor_lr;
  a.lr_c = c->cfg.critic_lr;
  a.eps = c->cfg.epsilon;
  a.slots = c->slots_src ? c->slots_src : c->d_slots;
  if (rb) {
    a.rs = rb->rs;
    a.ra = rb->ra;
    a.rr = rb->rr;
    a.rt = rb->rt;
    a.rs2 = rb->rs2;
    a.rsd = rb->rsd;
    a.rs2d = rb->rs2d;
    a.rrd = rb->rrd;
  }
  a.mean = c->has_scaler ? c->dmean : nullptr;
  a.sdev = c->has_scaler ? c->dscale : nullptr;
  a.theta = c->theta;
  a.grad = c->grad;
  a.target = c->target;
  a.adam_m = c->adam_m;
  a.adam_v = c->adam_v;
  a.whT = c->sb_whT;
  a.w2T = c->sb_w2T;
  a.sv = c->sb_sv;
  a.pw = c->dpw;
  a.alpha = c->sb_misc;
  a.stat_part = c->sb_misc + 4;
  a.stats = c->dstats;
  a.acc = c->dacc;
  a.aW1 = L.a[AW1].off;
  a.ab1 = L.a[AB1].off;
  a.aW2 = L.a[AW2].off;
  a.ab2 = L.a[AB2].off;
  a.aW3 = L.a[AW3].off;
  a.cWs = L.c[CWS].off;
  a.cbs = L.c[CBS].off;
  a.cWa = L.c[CWA].off;
  a.cba = L.c[CBA].off;
  a.cWh = L.c[CWH].off;
  a.cbh = L.c[CBH].off;
  a.cWo = L.c[CWO].off;
  a.cbo = L.c[CBO].off;
  a.stamps = c->sb_stamps;
  // all workgroups on one XCD (one L2 streams the weights) while they fit its
  // 32 CUs: +3 % at C2 (profiles/r3/sb_xcd_ab_c2.txt)
  a.xstride = c->sb_xstride ? c->sb_xstride : (ceil_div(B, SB_R) <= 32 ? 8 : 1);
  return a;
}

// Small-batch learner step: 4 launches (small_batch.h); the gather from the
// replay ring is fused into the phase kernels (slots already in c->d_slots).
static void learner_step_small(ddpg_ctx* c, ddpg_replay* rb, int B, float inv_b) {
  const Layout& L = c->L;
  const SbArgs a = sb_args(c, rb, B, inv_b);
  const int G = ceil_div(B, SB_R);
  const long long nc = (long long)(L.critic_end - L.critic_begin);
  const long long na = (long long)(L.actor_end - L.actor_begin);
  const double row_bytes = (2.0 * c->S + c->A + 2) * 4.0;
  {
    ProfScope ps(c, "sb_phase1", 0, 4.0 * (double)G * (L.total + nc) + B * row_bytes);
    hipLaunchKernelGGL(sb_phase1_kernel, dim3(G * a.xstride), dim3(SB_NT), c->sb_smem, c->cur, a);
    HIP_TRY(hipGetLastError());
  }
  {
    ProfScope ps(c, "sb_wgrad_adam", 2.0 * B * nc, 32.0 * nc);
    const SbGradTab& t = c->sb_tab[1];
    hipLaunchKernelGGL(sb_wgrad_adam_kernel, dim3(t.t[t.n].tile0), dim3(SB_GT), 0, c->cur, a, t,
                       1, G);
    HIP_TRY(hipGetLastError());
  }
  {
    ProfScope ps(c, "sb_phase3", 0, 4.0 * (double)G * (L.total + na) + B * c->S * 4.0);
    hipLaunchKernelGGL(sb_phase3_kernel, dim3(G * a.xstride), dim3(SB_NT), c->sb_smem, c->cur, a);
    HIP_TRY(hipGetLastError());
  }
  {
    ProfScope ps(c, "sb_wgrad_adam", 2.0 * B * na, 32.0 * na);
    const SbGradTab& t = c->sb_tab[0];
    hipLaunchKernelGGL(sb_wgrad_adam_kernel, dim3(t.t[t.n].tile0), dim3(SB_GT), 0, c->cur, a, t,
                       0, G);
    HIP_TRY(hipGetLastError());
  }
}

static void gather_launch(ddpg_ctx* c, ddpg_replay* rb, int B);

// The fused learner step on this step's slots (c->d_slots): the small-batch
// path (gather fused) or gather + the large-batch GEMM path.
static bool takes_small(const ddpg_ctx* c, int B) {
  return c->sb_ok && c->world == 1 && !c->comm && B <= c->sb_max_b;
}

static void learner_step_any(ddpg_ctx* c, ddpg_replay* rb, int B, float inv_b) {
  if (takes_small(c, B)) {
    learner_step_small(c, rb, B, inv_b);
  } else {
    gather_launch(c, rb, B);
    learner_step_dev(c, B, inv_b);
  }
}

// ====================================================================== helpers
static void upload_rows(ddpg_ctx* c, float* dst, int ld, const float* src, int B, int cols) {
  if (B <= 0 || cols <= 0) return;
  HIP_TRY(hipMemcpy2DAsync(dst, (size_t)ld * 4, src, (size_t)cols * 4, (size_t)cols * 4, B,
                           hipMemcpyHostToDevice, c->stream));
  const Twin t = act_twin(c, dst);
  if (t.p) {  // the twin covers the padded rows (pads are zero in both)
    hipLaunchKernelGGL(twin_kernel, dim3(std::min(ceil_div(B * ld, 256), 2048)), dim3(256), 0,
                       c->stream, dst, (long long)B * ld, t.p, t.ps, c->hnp);
    HIP_TRY(hipGetLastError());
  }
}
static void download_rows(ddpg_ctx* c, float* dst, const float* src, int ld, int B, int cols) {
  if (B <= 0 || cols <= 0) return;
  HIP_TRY(hipMemcpy2DAsync(dst, (size_t)cols * 4, src, (size_t)ld * 4, (size_t)cols * 4, B,
                           hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
}

static void check_b(ddpg_ctx* c, int B) {
  if (B <= 0 || B > c->Bmax) throw einval("batch %d outside [1, %d]", B, c->Bmax);
}

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

static void ctx_free(ddpg_ctx* c) {
  if (!c) return;
  if (c->comm) ncclCommDestroy(c->comm);
  for (auto& r : c->prof_recs) {
    (void)hipEventDestroy(r.e0);
    (void)hipEventDestroy(r.e1);
  }
  for (auto e : c->ev_pool) (void)hipEventDestroy(e);
  for (int i = 0; i < kSlotRing; ++i)
    if (c->slot_ev[i]) (void)hipEventDestroy(c->slot_ev[i]);
  if (c->h_slots) (void)hipHostFree(c->h_slots);
  if (c->h_pred) (void)hipHostFree(c->h_pred);
  for (auto& g : c->gslot) {
    if (g.exec) (void)hipGraphExecDestroy(g.exec);
    if (g.h_idx) (void)hipHostFree(g.h_idx);
    if (g.done) (void)hipEventDestroy(g.done);
  }
  if (c->step_done) (void)hipEventDestroy(c->step_done);
  for (void* p : {(void*)c->sb_save, (void*)c->sb_misc, (void*)c->sb_whT, (void*)c->sb_w2T,
                  (void*)c->sb_stamps})
    if (p) (void)hipFree(p);
  for (void* p : {(void*)c->atw, (void*)c->wtw, (void*)c->kc_part, (void*)c->kc_ticket})
    if (p) (void)hipFree(p);
  for (void* p : {(void*)c->dparams, (void*)c->dpw, (void*)c->dact, (void*)c->d_slots,
                  (void*)c->dmean, (void*)c->dscale, (void*)c->dacc, (void*)c->dstats_all})
    if (p) (void)hipFree(p);
  for (auto st : c->aux)
    if (st) (void)hipStreamDestroy(st);
  for (auto ev : c->fj)
    if (ev) (void)hipEventDestroy(ev);
  for (auto ev : c->cev)
    if (ev) (void)hipEventDestroy(ev);
  if (c->cs) (void)hipStreamDestroy(c->cs);
  if (c->stream && c->own_stream) (void)hipStreamDestroy(c->stream);
  delete c;
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

// ====================================================================== C ABI
extern "C" {

int ddpg_abi_version(void) { return DDPG_ABI_VERSION; }
const char* ddpg_global_error(void) { return g_err.c_str(); }
const char* ddpg_last_error(ddpg_ctx* c) { return c ? c->err.c_str() : g_err.c_str(); }

int ddpg_create(const ddpg_cfg* cfg, ddpg_ctx** out) {
  if (!cfg || !out) {
    g_err = "null argument";
    return DDPG_EINVAL;
  }
  ddpg_ctx* c = new ddpg_ctx();
  memset(c->slot_ev, 0, sizeof c->slot_ev);
  int rc = guard(c, [&] {
    const ddpg_cfg& k = *cfg;
    if (k.state_dim <= 0 || k.action_dim <= 0 || k.h1 <= 0 || k.h2 <= 0 || k.batch_max <= 0 ||
        k.critic_h1 < 0 || k.critic_h2 < 0)
      throw einval("dims must be positive (S=%d A=%d H1=%d H2=%d Bmax=%d)", k.state_dim,
                   k.action_dim, k.h1, k.h2, k.batch_max);
    if (k.action_dim > PROJ_MAX) throw einval("action_dim %d > %d", k.action_dim, PROJ_MAX);
    if (k.dtype != DDPG_FP32 && k.dtype != DDPG_BF16) throw einval("bad dtype %d", k.dtype);
    c->cfg = k;
    c->S = k.state_dim;
    c->A = k.action_dim;
    c->AH1 = k.h1;
    c->AH2 = k.h2;
    c->CH1 = k.critic_h1 > 0 ? k.critic_h1 : k.h1;
    c->CH2 = k.critic_h2 > 0 ? k.critic_h2 : k.h2;
    c->Bmax = k.batch_max;
    c->world = std::max(1, k.world);
    c->rank = k.rank;
    // bf16 twins: the bf16 configuration always; fp32 contexts keep exact
    // three-plane twins unless env DDPG_GEMM_H=0 / DDPG_GEMM=f32
    {
      const char* gh = getenv("DDPG_GEMM_H");
      const char* gf = getenv("DDPG_GEMM");
      const bool off_h = (gh && atoi(gh) == 0) || (gf && strcmp(gf, "f32") == 0);
      c->hnp = k.dtype == DDPG_BF16 ? 1 : (off_h ? 0 : 3);
    }
    // bf16 configuration: state / action rows padded with zeros to whole
    // k-tiles (64) / thin-K steps (8), so the first layers run K-padded
    // (K = S = 376 on gemm_h, K = A = 17 on thin_k)
    c->ldS = c->hnp == 1 ? rup(c->S, 64) : rup(c->S, 4);
    c->ldA = c->hnp == 1 ? rup(c->A, 8) : rup(c->A, 4);
    c->ldAH1 = rup(c->AH1, 4);
    c->ldAH2 = rup(c->AH2, 4);
    c->ldCH2 = rup(c->CH2, 4);
    c->ldC = rup(2 * c->CH1, 4);
    c->L.build(c->S, c->A, c->AH1, c->AH2, c->CH1, c->CH2);
    HIP_TRY(hipSetDevice(k.device));
    HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    c->cur = c->stream;
    for (auto& st : c->aux) HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    for (auto& ev : c->fj) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const size_t PT = c->L.total;
    HIP_TRY(hipMalloc(&c->dparams, 5 * PT * sizeof(float)));
    HIP_TRY(hipMemset(c->dparams, 0, 5 * PT * sizeof(float)));
    c->theta = c->dparams;
    c->target = c->dparams + PT;
    c->adam_m = c->dparams + 2 * PT;
    c->adam_v = c->dparams + 3 * PT;
    c->grad = c->dparams + 4 * PT;
    HIP_TRY(hipMalloc(&c->dpw, 64));
    {
      float pw[8] = {k.beta1, k.beta2, k.beta1, k.beta2, 0, 0, 0, 0};
      HIP_TRY(hipMemcpy(c->dpw, pw, sizeof pw, hipMemcpyHostToDevice));
    }
    c->dcounter = reinterpret_cast<unsigned*>(c->dpw + 4);
    c->dstats = c->dpw + 6;
    HIP_TRY(hipMalloc(&c->dacc, 4 * sizeof(double)));
    HIP_TRY(hipMemset(c->dacc, 0, 4 * sizeof(double)));

    // activation workspace
    const size_t B = (size_t)c->Bmax;
    const int NTP = std::max(ceil_div(c->AH2, 64), ceil_div(c->CH1, 64));
    const int NTQ = ceil_div(c->CH2, 64);
    const int mt = ceil_div(c->Bmax, std::min(64, TK_ROWS));  // row blocks of colsum partials
    const int nchunk = ceil_div(c->Bmax, std::min(kHeadRows, kHeadRows4));
    if (const char* mb = getenv("DDPG_GEMM_MIN_BLOCKS")) g_min_blocks = std::max(1, atoi(mb));
    {
      auto env_is = [](const char* name, const char* val) {
        const char* v = getenv(name);
        return v && strcmp(v, val) == 0;
      };
      c->sw.gemm_h = !env_is("DDPG_GEMM_H", "0");
      c->sw.gemm_s3 = !env_is("DDPG_GEMM", "f32");
      c->sw.thin_k = !env_is("DDPG_THINK", "0");
      c->sw.gemm_mf = env_is("DDPG_GEMM_MF", "32") ? 32 : 16;
      c->sw.gemm_h3 = !env_is("DDPG_GEMM_H3", "0");
      if (const char* v = getenv("DDPG_GEMM256")) c->sw.gemm256 = std::min(4, std::max(0, atoi(v)));
      c->sw.xcd = env_is("DDPG_XCD", "0") ? 0 : 1;
      c->sw.xcd_rect = !env_is("DDPG_XCD_RECT", "0");
      c->sw.skinny = !env_is("DDPG_SKINNY", "0");
      c->sw.l1_batch = !env_is("DDPG_L1BATCH", "0");
      c->sw.act_planes = !env_is("DDPG_ACT32", "1");
      c->sw.slots_h2d = env_is("DDPG_SLOTS_H2D", "1");
      if (const char* v = getenv("DDPG_TK_RPB")) c->sw.tk_rpb = std::max(0, atoi(v));
      c->sw.kcomb = !env_is("DDPG_KCOMB", "0");
      if (const char* v = getenv("DDPG_KCOMB_BLOCKS"))
        c->sw.kc_blocks = std::min(kKcTickets, std::max(1, atoi(v)));
      if (const char* v = getenv("DDPG_TEST_CS_SPIN")) c->test_cs_spin = std::max(0, atoi(v));
      if (env_is("DDPG_GRAPH_COMM", "0")) c->comm_graph = false;
    }
    c->split_cap_W1 = make_plan(c->S, c->AH1, c->Bmax, 0).splits;
    c->split_cap_W2 = make_plan(c->AH1, c->AH2, c->Bmax, 0).splits;
    c->split_cap_W3 = make_plan(c->AH2, c->A, c->Bmax, 0).splits;
    c->split_cap_Ws = make_plan(c->S, c->CH1, c->Bmax, 0).splits;
    c->split_cap_Wa = make_plan(c->A, c->CH1, c->Bmax, 0).splits;
    c->split_cap_Wh = make_plan(2 * c->CH1, c->CH2, c->Bmax, 0).splits;
    if (c->cfg.dtype == DDPG_BF16) {  // the 256 x 256-tile kernel splits finer
      auto cap256 = [&](int M, int N) {
        return (M % H2_BM || N % H2_BN) ? 1 : std::max(1, 256 / ((M / H2_BM) * (N / H2_BN)));
      };
      c->split_cap_W2 = std::max(c->split_cap_W2, cap256(c->AH1, c->AH2));
      c->split_cap_Wh = std::max(c->split_cap_Wh, cap256(2 * c->CH1, c->CH2));
    }
    struct Req {
      float** p;
      size_t n;
    };
    std::vector<Req> req = {
        {&c->s, B * c->ldS},   {&c->s2, B * c->ldS},   {&c->a, B * c->ldA},
        {&c->r, B},            {&c->t, B},             {&c->y, B},
        {&c->q, B},            {&c->dq, B},            {&c->th1, B * c->ldAH1},
        {&c->tcat, B * c->ldC}, {&c->ta2, B * c->ldA}, {&c->cat, B * c->ldC},
        {&c->h, B * c->ldCH2},  {&c->dhp, B * c->ldCH2}, {&c->dcat, B * c->ldC},
        {&c->h1, B * c->ldAH1}, {&c->h2, B * c->ldAH2},  {&c->o, B * c->ldA},
        {&c->mu, B * c->ldA},  {&c->cat2, B * c->ldC}, {&c->dhp2, B * c->ldCH2},
        {&c->da, B * c->ldA},  {&c->dz3, B * c->ldA},  {&c->dz2, B * c->ldAH2},
        {&c->dz1, B * c->ldAH1}, {&c->dain, B * c->A},
        {&c->ppart, (size_t)NTP * B * PROJ_MAX},
        {&c->qpart, (size_t)NTQ * B},
        {&c->ppart_t, (size_t)NTP * B * PROJ_MAX},
        {&c->qpart_t, (size_t)NTQ * B},
        {&c->colpart, (size_t)mt * std::max(2 * c->CH1, c->AH2 + c->AH1)},
        {&c->headpart, (size_t)nchunk * (2 * c->CH2 + 1)},
        {reinterpret_cast<float**>(&c->lpart), 2 * (size_t)ceil_div(c->Bmax, 256)},
        {&c->slab_W1, (size_t)c->split_cap_W1 * c->S * c->AH1},
        {&c->slab_W2, (size_t)c->split_cap_W2 * c->AH1 * c->AH2},
        {&c->slab_W3, (size_t)c->split_cap_W3 * c->AH2 * c->A},
        {&c->slab_Ws, (size_t)c->split_cap_Ws * c->S * c->CH1},
        {&c->slab_Wa, (size_t)c->split_cap_Wa * c->A * c->CH1},
        {&c->slab_Wh, (size_t)c->split_cap_Wh * 2 * c->CH1 * c->CH2},
    };
    size_t tot = 0;
    for (auto& r : req) tot += (r.n + 63) / 64 * 64;
    HIP_TRY(hipMalloc(&c->dact, tot * sizeof(float)));
    HIP_TRY(hipMemset(c->dact, 0, tot * sizeof(float)));
    size_t off = 0;
    for (auto& r : req) {
      *r.p = c->dact + off;
      off += (r.n + 63) / 64 * 64;
    }
    if (c->hnp) {
      c->act_n = tot;
      HIP_TRY(hipMalloc(&c->atw, tot * c->hnp * sizeof(__bf16)));
      HIP_TRY(hipMemset(c->atw, 0, tot * c->hnp * sizeof(__bf16)));
      HIP_TRY(hipMalloc(&c->wtw, 2 * PT * c->hnp * sizeof(__bf16)));
      // the GEMM operands among the activations (gemm_h.h needs rows on
      // 16-B boundaries: ld % 8 == 0)
      // w: the logical width.  Epilogue-written twins (w > 0) need it in whole
      // 8-column groups, so the twin stores never reach the row padding; s / s2
      // (w = 0) get their twins from the gather / upload, pads included.
      const struct {
        float* p;
        int ld, w;
      } tw[] = {{c->s, c->ldS, 0},           {c->s2, c->ldS, 0},
                {c->h1, c->ldAH1, c->AH1},   {c->th1, c->ldAH1, c->AH1},
                {c->cat, c->ldC, 2 * c->CH1}, {c->tcat, c->ldC, 2 * c->CH1},
                {c->cat2, c->ldC, 2 * c->CH1}, {c->dhp, c->ldCH2, c->CH2},
                {c->dhp2, c->ldCH2, c->CH2}, {c->dz2, c->ldAH2, c->AH2},
                {c->dz1, c->ldAH1, c->AH1},  {c->dcat, c->ldC, 2 * c->CH1}};
      for (const auto& t : tw) {
        // dz1 / dcat are read as twins only by the dW1 / dWs GEMMs (M = S):
        // below 128 state columns those never take the twin GEMM (and at
        // S <= 64 they run on the skinny kernel), so no twin is written
        if ((t.p == c->dz1 || t.p == c->dcat) && c->S < 128) continue;
        if (t.ld % 8 == 0 && t.w % 8 == 0) c->twinned.push_back({t.p, B * (size_t)t.ld});
      }
    }
    HIP_TRY(hipMalloc(&c->d_slots, B * sizeof(int)));
    HIP_TRY(hipHostMalloc(&c->h_slots, kSlotRing * B * sizeof(int)));
    for (int i = 0; i < kSlotRing; ++i) HIP_TRY(hipEventCreateWithFlags(&c->slot_ev[i], hipEventDisableTiming));
    c->idx_tmp.resize(B * c->world);
    for (auto& g : c->gslot) {
      HIP_TRY(hipHostMalloc(&g.h_idx, B * sizeof(int)));
      HIP_TRY(hipEventCreateWithFlags(&g.done, hipEventDisableTiming));
    }
    HIP_TRY(hipEventCreateWithFlags(&c->step_done, hipEventDisableTiming));
    if (const char* gv = getenv("DDPG_GRAPH")) c->use_graph = atoi(gv) != 0;
    if (const char* gv = getenv("DDPG_GRAPH_AUTO")) c->graph_auto = atoi(gv) != 0;
    if (const char* pv = getenv("DDPG_PAR")) c->par = atoi(pv) != 0;
    if (c->hnp && c->sw.kcomb) {
      // a combined launch has S x tiles < 256 + kc_blocks blocks of BM x 128
      // partials; two buffers suffice on one stream, eight cover the
      // concurrent branches of DDPG_PAR=1
      const int BMh = c->hnp == 1 ? 256 : 128;
      c->kc_rot = c->par ? 8 : 2;
      c->kc_part_n = (size_t)(256 + c->sw.kc_blocks) * BMh * HG_BN;
      HIP_TRY(hipMalloc(&c->kc_part, c->kc_rot * c->kc_part_n * sizeof(float)));
      HIP_TRY(hipMalloc(&c->kc_ticket, (size_t)c->kc_rot * kKcTickets * sizeof(unsigned)));
      HIP_TRY(hipMemset(c->kc_ticket, 0, (size_t)c->kc_rot * kKcTickets * sizeof(unsigned)));
    }
    {
      const int hmax = std::max(std::max(c->AH1, c->AH2), std::max(c->CH1, c->CH2));
      const int LX = rup(std::max(c->S, c->A), 4);
      const int LW = rup(std::max(std::max(c->AH1, c->AH2), std::max(2 * c->CH1, c->CH2)), 4);
      const size_t smem = sb_smem_floats(LX, LW) * sizeof(float);
      // vector weight streams need 4-aligned widths; 160 KiB of LDS per workgroup
      bool ok = c->world == 1 && hmax <= SB_MAXH && c->AH1 % 4 == 0 && c->AH2 % 4 == 0 &&
                c->CH1 % 4 == 0 && c->CH2 % 4 == 0 && smem <= 160 * 1024;
      if (const char* sv = getenv("DDPG_SMALL")) ok = ok && atoi(sv) != 0;
      if (ok) {
        c->sb_max_b = std::min(c->Bmax, 512);
        c->sb_smem = smem;
        if (const char* xv = getenv("DDPG_SB_XCD")) c->sb_xstride = atoi(xv) ? 8 : 1;
        const int G = ceil_div(c->sb_max_b, SB_R);
        const size_t Bp = (size_t)rup(c->sb_max_b, 4);
        // saved tensors, feature-major [width][Bp]: xs xa cat dcat h dhp dq h1 h2 dz1 dz2 dz3
        const size_t widths[12] = {(size_t)c->S, (size_t)c->A, 2 * (size_t)c->CH1,
                                   2 * (size_t)c->CH1, (size_t)c->CH2, (size_t)c->CH2, 1,
                                   (size_t)c->AH1, (size_t)c->AH2, (size_t)c->AH1,
                                   (size_t)c->AH2, (size_t)c->A};
        size_t tot = 0;
        for (size_t w : widths) tot += (Bp * w + 63) / 64 * 64;
        HIP_TRY(hipMalloc(&c->sb_save, tot * sizeof(float)));
        HIP_TRY(hipMemset(c->sb_save, 0, tot * sizeof(float)));
        float* ptrs[12];
        size_t off = 0;
        for (int k = 0; k < 12; ++k) {
          ptrs[k] = c->sb_save + off;
          off += (Bp * widths[k] + 63) / 64 * 64;
        }
        SbSave& sv = c->sb_sv;
        sv.Bp = (int)Bp;
        sv.xs = ptrs[0];
        sv.xa = ptrs[1];
        sv.cat = ptrs[2];
        sv.dcat = ptrs[3];
        sv.h = ptrs[4];
        sv.dhp = ptrs[5];
        sv.dq = ptrs[6];
        sv.h1 = ptrs[7];
        sv.h2 = ptrs[8];
        sv.dz1 = ptrs[9];
        sv.dz2 = ptrs[10];
        sv.dz3 = ptrs[11];
        const Layout& L = c->L;
        const int bp = (int)Bp;
        auto add = [bp](SbGradTab& t, const Tensor& ts, const float* X, const float* dY) {
          SbGradT& e = t.t[t.n];
          e.off = (long long)ts.off;
          e.K = ts.cols == 1 && X == nullptr ? 1 : ts.rows;
          e.N = ts.cols == 1 && X == nullptr ? ts.rows : ts.cols;
          e.X = X;
          e.ldx = bp;
          e.dY = dY;
          e.ldy = bp;
          int tn = 1;
          while (tn < e.N && tn < 64) tn *= 2;
          e.TN = tn;
          e.TK = SB_GT / tn;
          e.tile0 = t.n ? t.t[t.n - 1].tile0 + ceil_div(t.t[t.n - 1].K, t.t[t.n - 1].TK) *
                                                   ceil_div(t.t[t.n - 1].N, t.t[t.n - 1].TN)
                        : 0;
          ++t.n;
        };
        auto close = [](SbGradTab& t) {  // sentinel: t.t[t.n].tile0 = total tiles
          const SbGradT& l = t.t[t.n - 1];
          t.t[t.n].tile0 = l.tile0 + ceil_div(l.K, l.TK) * ceil_div(l.N, l.TN);
        };
        SbGradTab& ta = c->sb_tab[0];  // actor (networks.py:39-47)
        ta.n = 0;
        add(ta, L.a[AW1], sv.xs, sv.dz1);
        add(ta, L.a[AB1], nullptr, sv.dz1);
        add(ta, L.a[AW2], sv.h1, sv.dz2);
        add(ta, L.a[AB2], nullptr, sv.dz2);
        add(ta, L.a[AW3], sv.h2, sv.dz3);
        close(ta);
        ta.shadow = 2;
        SbGradTab& tc = c->sb_tab[1];  // critic (networks.py:130-137)
        tc.n = 0;
        add(tc, L.c[CWS], sv.xs, sv.dcat);
        add(tc, L.c[CBS], nullptr, sv.dcat);
        add(tc, L.c[CWA], sv.xa, sv.dcat + (size_t)c->CH1 * Bp);
        add(tc, L.c[CBA], nullptr, sv.dcat + (size_t)c->CH1 * Bp);
        add(tc, L.c[CWH], sv.cat, sv.dhp);
        add(tc, L.c[CBH], nullptr, sv.dhp);
        add(tc, L.c[CWO], sv.h, sv.dq);
        add(tc, L.c[CBO], nullptr, sv.dq);
        close(tc);
        tc.shadow = 4;
        HIP_TRY(hipMalloc(&c->sb_misc, (4 + 2 * (size_t)G) * sizeof(float)));
        HIP_TRY(hipMemset(c->sb_misc, 0, (4 + 2 * (size_t)G) * sizeof(float)));
        HIP_TRY(hipMalloc(&c->sb_whT, (size_t)2 * c->CH1 * c->CH2 * sizeof(float)));
        HIP_TRY(hipMalloc(&c->sb_w2T, (size_t)c->AH1 * c->AH2 * sizeof(float)));
        ta.sh = c->sb_w2T;
        tc.sh = c->sb_whT;
        HIP_TRY(hipFuncSetAttribute((const void*)sb_phase1_kernel,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
        HIP_TRY(hipFuncSetAttribute((const void*)sb_phase3_kernel,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
        HIP_TRY(hipFuncSetAttribute((const void*)sb_actor_predict_kernel,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
        HIP_TRY(hipHostMalloc(&c->h_pred, (size_t)c->Bmax * c->A * sizeof(float)));
        c->sb_ok = true;
        if (const char* st = getenv("DDPG_SB_STAMPS"))
          if (atoi(st)) {
            HIP_TRY(hipMalloc(&c->sb_stamps, 64 * sizeof(unsigned long long)));
            HIP_TRY(hipMemset(c->sb_stamps, 0, 64 * sizeof(unsigned long long)));
          }
      }
    }
    HIP_TRY(hipFuncSetAttribute((const void*)skinny_wgrad_kernel<8>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, sk_lds_bytes(8)));
    HIP_TRY(hipFuncSetAttribute((const void*)skinny_wgrad_kernel<16>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, sk_lds_bytes(16)));
    HIP_TRY(hipDeviceSynchronize());
  });
  if (rc != DDPG_OK) {
    ctx_free(c);
    *out = nullptr;
    return rc;
  }
  *out = c;
  return DDPG_OK;
}

void ddpg_destroy(ddpg_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->cfg.device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  ctx_free(c);
}

int ddpg_sync(ddpg_ctx* c) {
  return guard(c, [&] {
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->sb_stamps) {  // diagnostic: per-op cycle counts of the last small-batch step
      unsigned long long t[64];
      HIP_TRY(hipMemcpy(t, c->sb_stamps, sizeof t, hipMemcpyDeviceToHost));
      fprintf(stderr, "[sb stamps] phase1:");
      for (int i = 1; i <= 10; ++i) fprintf(stderr, " %llu", t[i] - t[i - 1]);
      fprintf(stderr, " total %llu | phase3:", t[10] - t[0]);
      for (int i = 33; i <= 42; ++i) fprintf(stderr, " %llu", t[i] - t[i - 1]);
      fprintf(stderr, " total %llu | wgrad c:", t[42] - t[32]);
      for (int i = 49; i <= 50; ++i) fprintf(stderr, " %llu", t[i] - t[i - 1]);
      fprintf(stderr, " | wgrad a:");
      for (int i = 57; i <= 58; ++i) fprintf(stderr, " %llu", t[i] - t[i - 1]);
      fprintf(stderr, "\n");
    }
  });
}

int ddpg_set_stream(ddpg_ctx* c, void* s) {
  return guard(c, [&] {
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->own_stream) HIP_TRY(hipStreamDestroy(c->stream));
    if (s) {
      c->stream = (hipStream_t)s;
      c->own_stream = false;
    } else {
      HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
      c->own_stream = true;
    }
    c->cur = c->stream;
  });
}

// ---------------------------------------------------------------- parameters
static void which_tensors(ddpg_ctx* c, int which, const Tensor** ts, int* nt, float** base) {
  const bool actor = which == DDPG_ACTOR || which == DDPG_ACTOR_TARGET ||
                     which == DDPG_ACTOR_ADAM_M || which == DDPG_ACTOR_ADAM_V ||
                     which == DDPG_ACTOR_GRAD;
  *ts = actor ? c->L.a : c->L.c;
  *nt = actor ? NA : NC;
  switch (which) {
    case DDPG_ACTOR:
    case DDPG_CRITIC: *base = c->theta; break;
    case DDPG_ACTOR_TARGET:
    case DDPG_CRITIC_TARGET: *base = c->target; break;
    case DDPG_ACTOR_ADAM_M:
    case DDPG_CRITIC_ADAM_M: *base = c->adam_m; break;
    case DDPG_ACTOR_ADAM_V:
    case DDPG_CRITIC_ADAM_V: *base = c->adam_v; break;
    case DDPG_ACTOR_GRAD:
    case DDPG_CRITIC_GRAD: *base = c->grad; break;
    default: throw einval("bad parameter set %d", which);
  }
}

int ddpg_param_count(ddpg_ctx* c, int which, size_t* n) {
  return guard(c, [&] {
    const Tensor* ts;
    int nt;
    float* base;
    which_tensors(c, which, &ts, &nt, &base);
    size_t tot = 0;
    for (int i = 0; i < nt; ++i) tot += ts[i].count();
    *n = tot;
  });
}

int ddpg_set_params(ddpg_ctx* c, int which, const float* host, size_t n) {
  return guard(c, [&] {
    if (which == DDPG_ACTOR_GRAD || which == DDPG_CRITIC_GRAD)
      throw einval("param set %d (gradient) is get-only", which);
    const Tensor* ts;
    int nt;
    float* base;
    which_tensors(c, which, &ts, &nt, &base);
    size_t tot = 0;
    for (int i = 0; i < nt; ++i) tot += ts[i].count();
    if (n != tot) throw einval("param set %d expects %zu floats, got %zu", which, tot, n);
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->sb_shadow_ok = false;
    c->wtw_ok = false;
    size_t o = 0;
    for (int i = 0; i < nt; ++i) {
      HIP_TRY(hipMemcpy(base + ts[i].off, host + o, ts[i].count() * 4, hipMemcpyHostToDevice));
      o += ts[i].count();
    }
  });
}

int ddpg_get_params(ddpg_ctx* c, int which, float* host, size_t n) {
  return guard(c, [&] {
    const Tensor* ts;
    int nt;
    float* base;
    which_tensors(c, which, &ts, &nt, &base);
    size_t tot = 0;
    for (int i = 0; i < nt; ++i) tot += ts[i].count();
    if (n != tot) throw einval("param set %d has %zu floats, buffer %zu", which, tot, n);
    HIP_TRY(hipStreamSynchronize(c->stream));
    size_t o = 0;
    for (int i = 0; i < nt; ++i) {
      HIP_TRY(hipMemcpy(host + o, base + ts[i].off, ts[i].count() * 4, hipMemcpyDeviceToHost));
      o += ts[i].count();
    }
  });
}

int ddpg_set_adam_powers(ddpg_ctx* c, int net, float b1p, float b2p) {
  return guard(c, [&] {
    if (net != 0 && net != 1) throw einval("net must be 0 (actor) or 1 (critic)");
    float pw[2] = {b1p, b2p};
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipMemcpy(c->dpw + 2 * net, pw, sizeof pw, hipMemcpyHostToDevice));
  });
}

int ddpg_get_adam_powers(ddpg_ctx* c, int net, float* b1p, float* b2p) {
  return guard(c, [&] {
    if (net != 0 && net != 1) throw einval("net must be 0 (actor) or 1 (critic)");
    float pw[2];
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipMemcpy(pw, c->dpw + 2 * net, sizeof pw, hipMemcpyDeviceToHost));
    *b1p = pw[0];
    *b2p = pw[1];
  });
}

int ddpg_set_scaler(ddpg_ctx* c, const double* mean, const double* scale, int S) {
  return guard(c, [&] {
    if (!mean || !scale) {
      c->has_scaler = false;
      return;
    }
    if (S != c->S) throw einval("scaler has %d features, state_dim is %d", S, c->S);
    if (!c->dmean) {
      HIP_TRY(hipMalloc(&c->dmean, S * sizeof(double)));
      HIP_TRY(hipMalloc(&c->dscale, S * sizeof(double)));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipMemcpy(c->dmean, mean, S * sizeof(double), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->dscale, scale, S * sizeof(double), hipMemcpyHostToDevice));
    c->has_scaler = true;
  });
}

// ---------------------------------------------------------------- 1:1 methods
int ddpg_actor_forward(ddpg_ctx* c, int target, const float* s, int B, float* a_out) {
  return guard(c, [&] {
    check_b(c, B);
    twins_refresh(c);
    if (c->sb_ok && B * c->S <= SB_PRED_MAX) {
      // action selection (ddpg.py:68-70): one launch, states in the kernel
      // arguments, result written to pinned host memory
      SbPredIn in;
      memcpy(in.s, s, sizeof(float) * B * c->S);
      const SbArgs a = sb_args(c, nullptr, B, 1.f);
      const size_t smem = (SB_RED + 2 * SB_BIAS + 8 * (size_t)a.LX + 8 * (size_t)a.LW) * 4;
      {
        ProfScope ps(c, "sb_actor_predict", 0, 0);
        hipLaunchKernelGGL(sb_actor_predict_kernel, dim3(ceil_div(B, SB_R)), dim3(SB_NT), smem,
                           c->stream, a, target ? c->target : c->theta, in, c->h_pred);
        HIP_TRY(hipGetLastError());
      }
      HIP_TRY(hipStreamSynchronize(c->stream));
      memcpy(a_out, c->h_pred, sizeof(float) * B * c->A);
      return;
    }
    upload_rows(c, c->s, c->ldS, s, B, c->S);
    actor_fwd(c, target ? c->target : c->theta, c->s, B, c->h1, nullptr, nullptr, c->mu);
    download_rows(c, a_out, c->mu, c->ldA, B, c->A);
  });
}

int ddpg_critic_forward(ddpg_ctx* c, int target, const float* s, const float* a, int B,
                        float* q_out) {
  return guard(c, [&] {
    check_b(c, B);
    twins_refresh(c);
    upload_rows(c, c->s, c->ldS, s, B, c->S);
    upload_rows(c, c->a, c->ldA, a, B, c->A);
    const float* base = target ? c->target : c->theta;
    const int nq = critic_fwd(c, base, c->s, c->a, B, c->cat, nullptr, 1, nullptr);
    hipLaunchKernelGGL(critic_q_kernel, dim3(ceil_div(B, 256)), dim3(256), 0, c->stream, c->qpart,
                       nq, B, P(c, base, c->L.c[CBO]), c->q, 0, nullptr,
                       nullptr, 0.f, nullptr);
    HIP_TRY(hipGetLastError());
    download_rows(c, q_out, c->q, 1, B, 1);
  });
}

int ddpg_critic_train(ddpg_ctx* c, const float* s, const float* a, const float* y, int B,
                      float* q_pre, float* loss) {
  return guard(c, [&] {
    check_b(c, B);
    twins_refresh(c);
    upload_rows(c, c->s, c->ldS, s, B, c->S);
    upload_rows(c, c->a, c->ldA, a, B, c->A);
    upload_rows(c, c->y, 1, y, B, 1);
    critic_train_dev(c, B, 1.0f / (float)(B * c->world), false);
    if (q_pre) download_rows(c, q_pre, c->q, 1, B, 1);
    if (loss) {
      float st[2];
      HIP_TRY(hipMemcpyAsync(st, c->dstats, sizeof st, hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      *loss = st[1];
    }
  });
}

int ddpg_critic_action_grad(ddpg_ctx* c, const float* s, const float* a, int B, float* da) {
  return guard(c, [&] {
    check_b(c, B);
    twins_refresh(c);
    upload_rows(c, c->s, c->ldS, s, B, c->S);
    upload_rows(c, c->a, c->ldA, a, B, c->A);
    critic_action_grad(c, c->s, c->a, B, c->da, nullptr, nullptr);
    download_rows(c, da, c->da, c->ldA, B, c->A);
  });
}

int ddpg_actor_train(ddpg_ctx* c, const float* s, const float* a_gradient, int B) {
  return guard(c, [&] {
    check_b(c, B);
    twins_refresh(c);
    upload_rows(c, c->s, c->ldS, s, B, c->S);
    // a_gradient as a single "partial" slab [1][B][A] for the dz3 finaliser
    HIP_TRY(hipMemcpyAsync(c->dain, a_gradient, (size_t)B * c->A * 4, hipMemcpyHostToDevice,
                           c->stream));
    actor_fwd(c, c->theta, c->s, B, c->h1, c->h2, c->o, c->mu);
    hipLaunchKernelGGL(action_grad_kernel, dim3(ceil_div(B * c->A, 256)), dim3(256), 0, c->stream,
                       c->dain, 1, B, c->A, B, c->o, c->ldA, c->cfg.action_scale, nullptr,
                       c->dz3);
    HIP_TRY(hipGetLastError());
    actor_train_dev(c, B, false);
    HIP_TRY(hipStreamSynchronize(c->stream));
  });
}

int ddpg_soft_update(ddpg_ctx* c, int mask) {
  return guard(c, [&] {
    twins_refresh(c);
    soft_update_dev(c, mask, 0);
    HIP_TRY(hipStreamSynchronize(c->stream));
  });
}

// ---------------------------------------------------------------- sampler
struct ddpg_sampler {
  Sampler s;
  explicit ddpg_sampler(int64_t seed) : s(seed) {}
};

int ddpg_sampler_create(int64_t seed, ddpg_sampler** out) {
  if (!out) return DDPG_EINVAL;
  *out = new ddpg_sampler(seed);
  return DDPG_OK;
}
void ddpg_sampler_destroy(ddpg_sampler* s) { delete s; }
int ddpg_sampler_sample(ddpg_sampler* s, int64_t n, int k, int64_t* out) {
  if (!s || !out || s->s.sample(n, k, out) != 0) {
    g_err = "sample larger than population or is negative";
    return DDPG_EINVAL;
  }
  return DDPG_OK;
}
int ddpg_sampler_getrandbits32(ddpg_sampler* s, uint32_t* out, int n) {
  if (!s || !out || n < 0) return DDPG_EINVAL;
  for (int i = 0; i < n; ++i) out[i] = s->s.rng.genrand_uint32();
  return DDPG_OK;
}

// ---------------------------------------------------------------- replay
static constexpr int kStageRows = 1024;

static int replay_create_impl(int device, int S, int A, int64_t cap, int64_t seed, int flags,
                              ddpg_replay** out) {
  if (!out) return DDPG_EINVAL;
  ddpg_replay* rb = new ddpg_replay(seed);
  int rc = rguard(rb, [&] {
    if (S <= 0 || A <= 0 || cap <= 0) throw einval("bad replay dims S=%d A=%d cap=%lld", S, A,
                                                   (long long)cap);
    if (flags & ~DDPG_REPLAY_F64) throw einval("bad replay flags %d", flags);
    rb->device = device;
    rb->S = S;
    rb->A = A;
    rb->cap = cap;
    rb->f64 = (flags & DDPG_REPLAY_F64) != 0;
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipStreamCreateWithFlags(&rb->stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&rb->last_read, hipEventDisableTiming));
    const size_t c = (size_t)cap, es = rb->es();
    void *ps, *ps2, *pr;
    HIP_TRY(hipMalloc(&ps, c * S * es));
    HIP_TRY(hipMalloc(&ps2, c * S * es));
    HIP_TRY(hipMalloc(&pr, c * es));
    if (rb->f64) {
      rb->rsd = (double*)ps;
      rb->rs2d = (double*)ps2;
      rb->rrd = (double*)pr;
    } else {
      rb->rs = (float*)ps;
      rb->rs2 = (float*)ps2;
      rb->rr = (float*)pr;
    }
    HIP_TRY(hipMalloc(&rb->ra, c * A * 4));
    HIP_TRY(hipMalloc(&rb->rt, c * 4));
    rb->st_s.resize((size_t)kStageRows * S * es);
    rb->st_s2.resize((size_t)kStageRows * S * es);
    rb->st_r.resize((size_t)kStageRows * es);
    rb->st_a.resize((size_t)kStageRows * A);
    rb->st_t.resize(kStageRows);
  });
  if (rc != DDPG_OK) {
    ddpg_replay_destroy(rb);
    *out = nullptr;
    return rc;
  }
  *out = rb;
  return DDPG_OK;
}

int ddpg_replay_create(int device, int S, int A, int64_t cap, int64_t seed, ddpg_replay** out) {
  return replay_create_impl(device, S, A, cap, seed, 0, out);
}

int ddpg_replay_create_ex(int device, int S, int A, int64_t cap, int64_t seed, int flags,
                          ddpg_replay** out) {
  return replay_create_impl(device, S, A, cap, seed, flags, out);
}

int ddpg_replay_is_f64(ddpg_replay* rb) { return rb && rb->f64 ? 1 : 0; }

void ddpg_replay_destroy(ddpg_replay* rb) {
  if (!rb) return;
  (void)hipSetDevice(rb->device);
  if (rb->stream) (void)hipStreamSynchronize(rb->stream);
  for (void* p : {(void*)rb->rs, (void*)rb->rs2, (void*)rb->rr, (void*)rb->rsd, (void*)rb->rs2d,
                  (void*)rb->rrd, (void*)rb->ra, (void*)rb->rt, (void*)rb->d_slots,
                  (void*)rb->d_tmp})
    if (p) (void)hipFree(p);
  if (rb->stream) (void)hipStreamDestroy(rb->stream);
  if (rb->last_read) (void)hipEventDestroy(rb->last_read);
  delete rb;
}

const char* ddpg_replay_last_error(ddpg_replay* rb) { return rb ? rb->err.c_str() : ""; }

// copy n consecutive insertions starting at insertion index `first` into the
// ring; s, s2, r are already in the ring's precision (rb->es() bytes each)
static void ring_write(ddpg_replay* rb, int64_t first, int n, const void* s, const float* a,
                       const void* r, const float* t, const void* s2) {
  const size_t es = rb->es(), S = rb->S, A = rb->A;
  const unsigned char* bs = (const unsigned char*)s;
  const unsigned char* bs2 = (const unsigned char*)s2;
  const unsigned char* br = (const unsigned char*)r;
  int done = 0;
  while (done < n) {
    const int64_t slot = (first + done) % rb->cap;
    const size_t run = (size_t)std::min<int64_t>(n - done, rb->cap - slot);
    HIP_TRY(hipMemcpyAsync(rb->ps() + slot * S * es, bs + done * S * es, run * S * es,
                           hipMemcpyHostToDevice, rb->stream));
    HIP_TRY(hipMemcpyAsync(rb->ps2() + slot * S * es, bs2 + done * S * es, run * S * es,
                           hipMemcpyHostToDevice, rb->stream));
    HIP_TRY(hipMemcpyAsync(rb->pr() + slot * es, br + done * es, run * es, hipMemcpyHostToDevice,
                           rb->stream));
    HIP_TRY(hipMemcpyAsync(rb->ra + slot * A, a + done * A, run * A * 4, hipMemcpyHostToDevice,
                           rb->stream));
    HIP_TRY(hipMemcpyAsync(rb->rt + slot, t + done, run * 4, hipMemcpyHostToDevice, rb->stream));
    done += (int)run;
  }
}

static void replay_flush(ddpg_replay* rb) {
  if (rb->st_n == 0) return;
  if (rb->last_read) HIP_TRY(hipStreamWaitEvent(rb->stream, rb->last_read, 0));
  ring_write(rb, rb->st_first, rb->st_n, rb->st_s.data(), rb->st_a.data(), rb->st_r.data(),
             rb->st_t.data(), rb->st_s2.data());
  HIP_TRY(hipStreamSynchronize(rb->stream));  // staging is reused after this
  rb->st_n = 0;
}

extern "C++" {
// n host values of type T into dst in the ring's precision (float or double)
template <class T>
static void to_ring(const ddpg_replay* rb, const T* src, size_t n, unsigned char* dst) {
  if (rb->f64) {
    double* d = (double*)dst;
    for (size_t i = 0; i < n; ++i) d[i] = (double)src[i];
  } else {
    float* d = (float*)dst;
    for (size_t i = 0; i < n; ++i) d[i] = (float)src[i];
  }
}

// ReplayBuffer.add for n rows whose s, s2, r are float (T = float) or float64
// (T = double); converted to the ring's precision on the host.
template <class T>
static void replay_add_impl(ddpg_replay* rb, const T* s, const float* a, const T* r,
                            const uint8_t* t, const T* s2, int n) {
  if (n < 0) throw einval("negative row count");
  if (n > 0 && (!s || !a || !r || !t || !s2)) throw einval("null row array");
  HIP_TRY(hipSetDevice(rb->device));
  const size_t S = rb->S, A = rb->A, es = rb->es();
  if (n >= kStageRows) {  // bulk insert
    replay_flush(rb);
    if (rb->last_read) HIP_TRY(hipStreamWaitEvent(rb->stream, rb->last_read, 0));
    // only the last `cap` rows can survive; skip the ones that would be overwritten
    const int64_t skip = n > rb->cap ? n - rb->cap : 0;
    const size_t m = (size_t)(n - skip);
    std::vector<float> tf(m);
    for (size_t i = 0; i < m; ++i) tf[i] = t[skip + i] ? 1.f : 0.f;
    const bool same = (sizeof(T) == es);  // caller's arrays already in ring precision
    std::vector<unsigned char> cs, cs2, cr;
    const void *ps = s + skip * S, *ps2 = s2 + skip * S, *pr = r + skip;
    if (!same) {
      cs.resize(m * S * es);
      cs2.resize(m * S * es);
      cr.resize(m * es);
      to_ring(rb, s + skip * S, m * S, cs.data());
      to_ring(rb, s2 + skip * S, m * S, cs2.data());
      to_ring(rb, r + skip, m, cr.data());
      ps = cs.data();
      ps2 = cs2.data();
      pr = cr.data();
    }
    ring_write(rb, rb->total + skip, (int)m, ps, a + skip * A, pr, tf.data(), ps2);
    HIP_TRY(hipStreamSynchronize(rb->stream));
    rb->total += n;
    rb->count = std::min<int64_t>(rb->total, rb->cap);
    return;
  }
  int done = 0;
  while (done < n) {
    if (rb->st_n == 0) rb->st_first = rb->total;
    const int take = std::min(n - done, kStageRows - rb->st_n);
    to_ring(rb, s + done * S, take * S, rb->st_s.data() + rb->st_n * S * es);
    to_ring(rb, s2 + done * S, take * S, rb->st_s2.data() + rb->st_n * S * es);
    to_ring(rb, r + done, take, rb->st_r.data() + rb->st_n * es);
    memcpy(rb->st_a.data() + rb->st_n * A, a + done * A, take * A * 4);
    for (int i = 0; i < take; ++i) rb->st_t[rb->st_n + i] = t[done + i] ? 1.f : 0.f;
    rb->st_n += take;
    rb->total += take;
    rb->count = std::min<int64_t>(rb->total, rb->cap);
    done += take;
    if (rb->st_n == kStageRows) replay_flush(rb);
  }
}
}  // extern "C++"

int ddpg_replay_add(ddpg_replay* rb, const float* s, const float* a, const float* r,
                    const uint8_t* t, const float* s2, int n) {
  return rguard(rb, [&] { replay_add_impl<float>(rb, s, a, r, t, s2, n); });
}

int ddpg_replay_add_f64(ddpg_replay* rb, const double* s, const float* a, const double* r,
                        const uint8_t* t, const double* s2, int n) {
  return rguard(rb, [&] { replay_add_impl<double>(rb, s, a, r, t, s2, n); });
}

int64_t ddpg_replay_size(ddpg_replay* rb) { return rb ? rb->count : 0; }
int64_t ddpg_replay_total_added(ddpg_replay* rb) { return rb ? rb->total : 0; }

int ddpg_replay_clear(ddpg_replay* rb) {
  return rguard(rb, [&] {
    HIP_TRY(hipStreamSynchronize(rb->stream));
    rb->count = rb->total = 0;
    rb->st_n = 0;
  });
}

// deque position -> ring slot (deque holds insertions [total-count, total))
static inline int pos_to_slot(const ddpg_replay* rb, int64_t pos) {
  return (int)((rb->total - rb->count + pos) % rb->cap);
}

extern "C++" {
// ReplayBuffer.sample_batch to host arrays of type T (s, s2, r).  The rows are
// gathered on device in the ring's own precision (byte copies) and converted
// on the host: exact for a float64 ring read as float64 and for a fp32 ring.
template <class T>
static int sample_impl(ddpg_replay* rb, int B, T* s, float* a, T* r, uint8_t* t, T* s2,
                       int64_t* idx_out) {
  int got = 0;
  int rc = rguard(rb, [&] {
    if (B < 0) throw einval("negative batch");
    HIP_TRY(hipSetDevice(rb->device));
    replay_flush(rb);
    const int k = (int)std::min<int64_t>(B, rb->count);  // replay_buffer.py:36-39
    rb->tmp_idx.resize(std::max(1, k));
    if (rb->sampler.sample(rb->count, k, rb->tmp_idx.data()) != 0) throw einval("sample failed");
    got = k;
    if (idx_out) memcpy(idx_out, rb->tmp_idx.data(), k * sizeof(int64_t));
    if (k == 0) return;
    rb->tmp_slot.resize(k);
    for (int i = 0; i < k; ++i) rb->tmp_slot[i] = pos_to_slot(rb, rb->tmp_idx[i]);
    const size_t S = rb->S, A = rb->A, es = rb->es();
    if (rb->d_slots_cap < k) {
      if (rb->d_slots) HIP_TRY(hipFree(rb->d_slots));
      HIP_TRY(hipMalloc(&rb->d_slots, k * sizeof(int)));
      rb->d_slots_cap = k;
    }
    const size_t row_bytes = 2 * S * es + A * 4 + es + 4;
    const size_t need = (size_t)k * row_bytes;
    if (rb->d_tmp_cap < need) {
      if (rb->d_tmp) HIP_TRY(hipFree(rb->d_tmp));
      HIP_TRY(hipMalloc(&rb->d_tmp, need));
      rb->d_tmp_cap = need;
    }
    // output planes, each [k][row bytes]: s | s2 | a | r | t
    unsigned char* o_s = rb->d_tmp;
    unsigned char* o_s2 = o_s + k * S * es;
    unsigned char* o_a = o_s2 + k * S * es;
    unsigned char* o_r = o_a + k * A * 4;
    unsigned char* o_t = o_r + k * es;
    HIP_TRY(hipMemcpyAsync(rb->d_slots, rb->tmp_slot.data(), k * sizeof(int),
                           hipMemcpyHostToDevice, rb->stream));
    struct Plane {
      const unsigned char* src;
      unsigned char* dst;
      size_t bytes;
    } planes[5] = {{rb->ps(), o_s, S * es},
                   {rb->ps2(), o_s2, S * es},
                   {(const unsigned char*)rb->ra, o_a, A * 4},
                   {rb->pr(), o_r, es},
                   {(const unsigned char*)rb->rt, o_t, 4}};
    for (const Plane& pl : planes) {
      hipLaunchKernelGGL(gather_bytes_kernel, dim3(std::min(ceil_div(k, 4), 4096)), dim3(256), 0,
                         rb->stream, rb->d_slots, k, pl.src, pl.dst, (long long)pl.bytes);
      HIP_TRY(hipGetLastError());
    }
    std::vector<unsigned char> tmp(need);
    HIP_TRY(hipMemcpyAsync(tmp.data(), rb->d_tmp, need, hipMemcpyDeviceToHost, rb->stream));
    HIP_TRY(hipStreamSynchronize(rb->stream));
    auto conv = [&](const unsigned char* src, size_t n, T* dst) {
      if (!dst) return;
      if (rb->f64)
        for (size_t i = 0; i < n; ++i) dst[i] = (T)((const double*)src)[i];
      else
        for (size_t i = 0; i < n; ++i) dst[i] = (T)((const float*)src)[i];
    };
    const size_t off_s2 = k * S * es, off_a = 2 * off_s2, off_r = off_a + k * A * 4,
                 off_t = off_r + k * es;
    conv(tmp.data(), k * S, s);
    conv(tmp.data() + off_s2, k * S, s2);
    conv(tmp.data() + off_r, k, r);
    if (a) memcpy(a, tmp.data() + off_a, (size_t)k * A * 4);
    if (t)
      for (int i = 0; i < k; ++i) t[i] = ((const float*)(tmp.data() + off_t))[i] != 0.f;
  });
  return rc == DDPG_OK ? got : rc;
}
}  // extern "C++"

int ddpg_replay_sample_batch(ddpg_replay* rb, int B, float* s, float* a, float* r, uint8_t* t,
                             float* s2, int64_t* idx_out) {
  return sample_impl<float>(rb, B, s, a, r, t, s2, idx_out);
}

int ddpg_replay_sample_batch_f64(ddpg_replay* rb, int B, double* s, float* a, double* r,
                                 uint8_t* t, double* s2, int64_t* idx_out) {
  return sample_impl<double>(rb, B, s, a, r, t, s2, idx_out);
}

// ---------------------------------------------------------------- fused step
static void gather_launch(ddpg_ctx* c, ddpg_replay* rb, int B) {
  ProfScope ps(c, "gather", 0, (double)B * (2.0 * c->S + c->A + 2) * 8.0);
  hipLaunchKernelGGL(gather_rows_kernel, dim3(ceil_div(B, 4)), dim3(256), 0, c->cur,
                     c->slots_src ? c->slots_src : c->d_slots, B, rb->rs, rb->ra, rb->rr, rb->rt,
                     rb->rs2, rb->rsd, rb->rs2d,
                     rb->rrd, c->S, c->A, c->s,
                     c->s2, c->ldS, c->a, c->ldA, c->r, c->t, c->has_scaler ? c->dmean : nullptr,
                     c->has_scaler ? c->dscale : nullptr, act_twin(c, c->s).p,
                     act_twin(c, c->s2).p, act_twin(c, c->s).ps, c->hnp);
  HIP_TRY(hipGetLastError());
}

static void step_common(ddpg_ctx* c, ddpg_replay* rb, const int64_t* idx, int Bg,
                        ddpg_stats* stats) {
  if (rb->S != c->S || rb->A != c->A)
    throw einval("replay dims (S=%d, A=%d) != network dims (S=%d, A=%d)", rb->S, rb->A, c->S,
                 c->A);
  if (Bg % c->world) throw einval("global batch %d not divisible by world %d", Bg, c->world);
  const int B = Bg / c->world;
  check_b(c, B);
  const int64_t* mine = idx + (size_t)c->rank * B;  // this rank's slice of the global draw
  const float inv_b = 1.0f / (float)Bg;
  const bool small = takes_small(c, B);
  sb_refresh_shadows(c);
  // the small path reads no twins: they are rebuilt lazily by the next
  // large-batch call (every 1:1 method and large step calls twins_refresh)
  if (!small) twins_refresh(c);
  // graphs: not profiling (per-kernel events stay eager); a data-parallel
  // step captures its RCCL calls as graph nodes (DDPG_GRAPH_COMM=0: eager)
  bool idle = true;  // the previous step has finished (never-recorded event: success)
  if (c->graph_auto && small) {
    const hipError_t q = hipEventQuery(c->step_done);
    if (q != hipSuccess && q != hipErrorNotReady) HIP_TRY(q);
    idle = q == hipSuccess;
  }
  const bool graph_ok = c->comm ? c->comm_graph : c->world == 1;
  bool graphed = false;
  if (c->use_graph && idle && graph_ok && !c->prof) {
    auto& g = c->gslot[c->gcur];
    HIP_TRY(hipEventSynchronize(g.done));  // this slot's previous replay has finished
    for (int i = 0; i < B; ++i) g.h_idx[i] = pos_to_slot(rb, mine[i]);
    if (!g.exec || g.B != B || g.rb != rb || g.scaler != c->has_scaler) {
      if (g.exec) HIP_TRY(hipGraphExecDestroy(g.exec));
      g.exec = nullptr;
      hipGraph_t graph = nullptr;
      HIP_TRY(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
      try {
        if (c->sw.slots_h2d) {
          HIP_TRY(hipMemcpyAsync(c->d_slots, g.h_idx, (size_t)B * sizeof(int),
                                 hipMemcpyHostToDevice, c->stream));
          c->slots_src = c->d_slots;
        } else {
          c->slots_src = g.h_idx;  // read in place by the replay (pinned; rewritten only
                                   // after this slot's previous replay is done)
        }
        learner_step_any(c, rb, B, inv_b);
        c->slots_src = nullptr;
        HIP_TRY(hipStreamEndCapture(c->stream, &graph));
        HIP_TRY(hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0));
        HIP_TRY(hipGraphDestroy(graph));
        graph = nullptr;
      } catch (const DdpgError& e) {
        c->slots_src = nullptr;
        hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(c->stream, &st) == hipSuccess && st != hipStreamCaptureStatusNone) {
          hipGraph_t dead = nullptr;
          (void)hipStreamEndCapture(c->stream, &dead);
          if (dead) (void)hipGraphDestroy(dead);
        }
        if (graph) (void)hipGraphDestroy(graph);
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
        g.exec = nullptr;
        (void)hipGetLastError();
        if (!c->comm) throw;
        // RCCL calls did not capture here: this ctx runs its steps eagerly
        c->comm_graph = false;
        c->cur = c->stream;
        c->td_nqt = 0;
        fprintf(stderr, "[ddpg] step graph with RCCL calls failed (%s); eager steps\n",
                e.msg.c_str());
      }
      if (g.exec) {
        g.B = B;
        g.rb = rb;
        g.scaler = c->has_scaler;
      }
    }
    if (g.exec) {
      c->gcur ^= 1;
      HIP_TRY(hipGraphLaunch(g.exec, c->stream));
      HIP_TRY(hipEventRecord(g.done, c->stream));
      graphed = true;
    }
  }
  if (!graphed) {
    const int si = c->slot_i;
    c->slot_i = (c->slot_i + 1) % kSlotRing;
    HIP_TRY(hipEventSynchronize(c->slot_ev[si]));
    int* hs = c->h_slots + (size_t)si * c->Bmax;
    for (int i = 0; i < B; ++i) hs[i] = pos_to_slot(rb, mine[i]);
    if (c->sw.slots_h2d) {
      HIP_TRY(hipMemcpyAsync(c->d_slots, hs, (size_t)B * sizeof(int), hipMemcpyHostToDevice,
                             c->stream));
      c->slots_src = c->d_slots;
    } else {
      c->slots_src = hs;  // read in place (pinned; reused kSlotRing steps later, after slot_ev)
    }
    try {
      learner_step_any(c, rb, B, inv_b);
    } catch (...) {
      c->slots_src = nullptr;
      throw;
    }
    c->slots_src = nullptr;
    HIP_TRY(hipEventRecord(c->slot_ev[si], c->stream));
  }
  HIP_TRY(hipEventRecord(rb->last_read, c->stream));
  HIP_TRY(hipEventRecord(c->step_done, c->stream));
  // Host-side state flags, updated here because a graph replay runs no host
  // code: a large-path step moved theta without refreshing the small path's
  // W^T shadows; a small-path step moved theta / target without their twins.
  if (small)
    c->wtw_ok = false;
  else
    c->sb_shadow_ok = false;
  if (stats) {
    float st[2];
    HIP_TRY(hipMemcpyAsync(st, c->dstats, sizeof st, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    stats->q_max = st[0];
    stats->loss = st[1];
  }
}

int ddpg_learner_step(ddpg_ctx* c, ddpg_replay* rb, int Bg, ddpg_stats* stats) {
  return guard(c, [&] {
    if (!rb) throw einval("null replay");
    replay_flush(rb);
    if (rb->count < Bg) throw einval("replay holds %lld rows < batch %d", (long long)rb->count, Bg);
    c->idx_tmp.resize(Bg);
    if (rb->sampler.sample(rb->count, Bg, c->idx_tmp.data()) != 0) throw einval("sample failed");
    step_common(c, rb, c->idx_tmp.data(), Bg, stats);
  });
}

int ddpg_learner_step_indices(ddpg_ctx* c, ddpg_replay* rb, const int64_t* idx, int Bg,
                              ddpg_stats* stats) {
  return guard(c, [&] {
    if (!rb || !idx) throw einval("null argument");
    replay_flush(rb);
    for (int i = 0; i < Bg; ++i)
      if (idx[i] < 0 || idx[i] >= rb->count) throw einval("index %lld out of range", (long long)idx[i]);
    step_common(c, rb, idx, Bg, stats);
  });
}

int ddpg_read_stats(ddpg_ctx* c, double* qsum, double* lsum, int64_t* steps, int reset) {
  return guard(c, [&] {
    double acc[4];
    HIP_TRY(hipMemcpyAsync(acc, c->dacc, sizeof acc, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (qsum) *qsum = acc[0];
    if (lsum) *lsum = acc[1];
    if (steps) *steps = (int64_t)acc[2];
    if (reset) HIP_TRY(hipMemsetAsync(c->dacc, 0, 4 * sizeof(double), c->stream));
  });
}

// ---------------------------------------------------------------- comm
// comm stream, its events and the stats all-gather buffer for a communicator
// of `cworld` ranks
static void comm_setup(ddpg_ctx* c, int cworld) {
  HIP_TRY(hipSetDevice(c->cfg.device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (!c->dstats_all) HIP_TRY(hipMalloc(&c->dstats_all, 2 * (size_t)cworld * sizeof(float)));
  if (!c->cs) HIP_TRY(hipStreamCreateWithFlags(&c->cs, hipStreamNonBlocking));
  for (auto& ev : c->cev)
    if (!ev) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
}

int ddpg_comm_unique_id(char* out128) {
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) {
    g_err = ncclGetErrorString(r);
    return DDPG_ECOMM;
  }
  static_assert(sizeof(id) == 128, "ncclUniqueId size");
  memcpy(out128, &id, 128);
  return DDPG_OK;
}

int ddpg_comm_init(ddpg_ctx* c, const char* id128, int world, int rank) {
  return guard(c, [&] {
    if (world != c->world || rank != c->rank)
      throw einval("comm (%d/%d) != cfg (%d/%d)", rank, world, c->rank, c->world);
    if (!id128) throw einval("null unique id");
    if (c->comm) throw DdpgError(DDPG_ESTATE, "communicator already initialised");
    // world == 1 makes a 1-rank communicator: the data-parallel exchange then
    // runs (as an identity) through the same RCCL call sites as world > 1
    ncclUniqueId id;
    memcpy(&id, id128, 128);
    comm_setup(c, world);
    nccl_try(ncclCommInitRank(&c->comm, world, id, rank));
    c->cworld = world;
  });
}

int ddpg_comm_init_proxy(ddpg_ctx* c) {
  return guard(c, [&] {
    if (c->comm) throw DdpgError(DDPG_ESTATE, "communicator already initialised");
    ncclUniqueId id;
    nccl_try(ncclGetUniqueId(&id));
    comm_setup(c, 1);
    nccl_try(ncclCommInitRank(&c->comm, 1, id, 0));
    c->cworld = 1;
  });
}

// ---------------------------------------------------------------- profiling
int ddpg_profile_enable(ddpg_ctx* c, int enable) {
  return guard(c, [&] {
    prof_collect(c);
    c->prof_agg.clear();
    c->prof = enable != 0;
  });
}

int ddpg_profile_read(ddpg_ctx* c, int n, char (*names)[64], double* ms, int64_t* launches,
                      double* flops, double* bytes) {
  int count = 0;
  int rc = guard(c, [&] {
    prof_collect(c);
    for (auto& kv : c->prof_agg) {
      if (count >= n) break;
      snprintf(names[count], 64, "%s", kv.first.c_str());
      ms[count] = kv.second.ms;
      launches[count] = kv.second.launches;
      flops[count] = kv.second.flops;
      bytes[count] = kv.second.bytes;
      ++count;
    }
  });
  return rc == DDPG_OK ? count : rc;
}

}  // extern "C"
