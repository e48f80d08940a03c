// The learner step (ddpg.py:86-113) from its building blocks: actor / critic
// forward, critic train, dQ/da, actor train, Adam + soft update, the fused
// step (gather, hipGraph capture and replay, the small-batch path) and the
// 1:1 reference methods of networks.py.  DESIGN.md §1, §4, §5.
#include <atomic>
#include <chrono>
#include <functional>
#include "ctx.h"
#include "kernels.h"
#include "small_batch.h"

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

// The actor's layer 2 (networks.py:57-60) with the W3 projection partials of
// the output layer in its epilogue (into c->ppart); h2 stored when non-null.
static GemmPlan actor_l2(ddpg_ctx* c, const float* base, int B, const float* h1, float* h2) {
  const Layout& L = c->L;
  GemmEpi e = epi_none();
  e.out = h2;
  e.ldo = c->ldAH2;
  e.bias = P(c, base, L.a[AB2]);
  e.act = 1;
  e.proj = P(c, base, L.a[AW3]);
  e.proj_n = c->A;
  e.proj_sn = c->A;
  e.proj_sa = 1;
  e.proj_out = c->ppart;
  return gemm_launch<L_RK, L_KR>(c, "fwd_head", h1, c->ldAH1, P(c, base, L.a[AW2]), c->AH2, B,
                                 c->AH2, c->AH1, e);
}

// o = tanh(sum of the nt projection partials in c->ppart), mu = scale o
// (networks.py:61-63)
static void actor_out_launch(ddpg_ctx* c, int nt, int B, float* o, float* mu) {
  ProfScope ps(c, "actor_out", 0, 0);
  hipLaunchKernelGGL(actor_out_kernel, dim3(ceil_div(B * c->A, 256)), dim3(256), 0, c->cur,
                     c->ppart, nt, B, c->A, c->cfg.action_scale, o, mu, c->ldA);
  HIP_TRY(hipGetLastError());
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
  const GemmPlan pl = actor_l2(c, base, B, h1, h2);
  actor_out_launch(c, pl.nt(c->AH2), B, o, mu);
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
  // cat2 (the critic at (s, mu), networks.py:143) with one bf16 plane: its
  // fp32 values are read only as the action half's EluGrad operand (the
  // action-gradient dX), so the state half writes its twin alone when the
  // hidden layer reads the twin
  if (!ct.p && cat == c->cat2 && c->hnp == 1 && c->sw.half_twin) {
    const Twin t2 = act_twin(c, cat);
    if (t2.p && gemm_h_ok<L_RK, L_KR>(c, cat, c->ldC, P(c, base, L.c[CWH]), c->CH2, B, c->CH2,
                                      2 * c->CH1, 1, &kh)) {
      tp[0].out = nullptr;
      tp[0].outh = t2.p;
      tp[0].hps = t2.ps;
      tp[0].hnp = c->hnp;
    }
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
      e.out = tp[0].out;  // as critic_l1_parts chose (fp32 and / or twin)
      e.outh = tp[0].outh;
      e.h_plane_stride = tp[0].outh ? tp[0].hps : ct.ps;
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

// TF ApplyAdam over one network's flat region.  advance: also advance its
// beta powers right after (1:1 API path).  soft (fused step): the same pass
// also soft-updates this network's targets from the new parameters and does
// its share of the beta-power bookkeeping (adam_hooks_for).
// fused learner step: the beta-power bookkeeping rides on the two passes
// (AdamHooks, kernels.h) -- the critic's pass runs first
static AdamHooks adam_hooks_for(ddpg_ctx* c, int net, bool fold) {
  AdamHooks h;
  memset(&h, 0, sizeof h);
  if (!fold) return h;
  float* alpha_slot = c->dpw + 8;
  if (net == 1) {
    h.pre_pw = c->dpw;
    h.pre_alpha = alpha_slot;
    h.pre_lr = c->cfg.actor_lr;
  } else {
    h.alpha_in = alpha_slot;
    h.adv_pw = c->dpw + 2;
  }
  return h;
}

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
                       c->hnp, soft ? c->target + b : nullptr, tau, omt, soft ? ttw : nullptr,
                       adam_hooks_for(c, net, soft));
    HIP_TRY(hipGetLastError());
  }
  if (advance) {
    hipLaunchKernelGGL(advance_powers_kernel, dim3(1), dim3(1), 0, c->cur, c->dpw, 1 << net,
                       c->cfg.beta1, c->cfg.beta2);
    HIP_TRY(hipGetLastError());
  }
}

// adam_launch with the network's gradient reduction (tab) folded into the
// same pass: no exchange sits between them (no communicator).  The table's
// slab segments plus direct segments for the rest of the network's region
// (gradients already written in place) cover it exactly once.
static void adam_reduce_launch(ddpg_ctx* c, int net, const ReduceTable& tab, bool advance,
                               bool soft) {
  const long long b = (long long)(net == 0 ? c->L.actor_begin : c->L.critic_begin);
  const long long e = (long long)(net == 0 ? c->L.actor_end : c->L.critic_end);
  float* G = c->grad;
  std::vector<const ReduceSeg*> segs;
  for (int i = 0; i < tab.nseg; ++i) segs.push_back(&tab.seg[i]);
  std::sort(segs.begin(), segs.end(),
            [](const ReduceSeg* x, const ReduceSeg* y) { return x->dst < y->dst; });
  AdamTable t;
  t.nseg = 0;
  int blocks = 0;
  double rbytes = 0;
  auto add = [&](const float* src, long long off, long long count, long long stride, int nslab,
                 bool v4) {
    if (count <= 0) return;
    if (t.nseg == ADAM_MAXSEG) throw DdpgError(DDPG_EINVAL, "adam_reduce: segment table full");
    AdamSeg& g = t.seg[t.nseg++];
    g.src = src;
    g.off = off;
    g.count = count;
    g.slab_stride = stride;
    g.nslab = nslab;
    // float4 also needs every flat array (theta, m, v, targets, twins) aligned at off
    g.vec4 = v4 && count % 4 == 0 && off % 4 == 0 && stride % 4 == 0 && aligned16(src);
    g.wg = src != G + off;
    const long long units = g.vec4 ? count / 4 : count;
    const int epb = 256 / slab_groups(nslab);
    g.nblk = (int)std::min<long long>(2048, (units + epb - 1) / epb);
    g.blk0 = blocks;
    blocks += g.nblk;
    if (g.wg) rbytes += 4.0 * count * (nslab + 1);
  };
  long long cur = b;
  for (const ReduceSeg* r : segs) {
    const long long off = (long long)(r->dst - G);
    if (off < cur || off + r->count > e)
      throw DdpgError(DDPG_EINVAL, "adam_reduce: gradient segments overlap or leave the network");
    add(G + cur, cur, off - cur, 0, 1, true);
    add(r->src, off, r->count, r->slab_stride, r->nslab, r->vec4 != 0);
    cur = off + r->count;
  }
  add(G + cur, cur, e - cur, 0, 1, true);
  const long long n = e - b;
  c->sb_shadow_ok = false;
  AdamArgs a;
  a.p = c->theta;
  a.m = c->adam_m;
  a.v = c->adam_v;
  a.g = G;
  a.pw = c->dpw + 2 * net;
  a.lr = net == 0 ? c->cfg.actor_lr : c->cfg.critic_lr;
  a.b1 = c->cfg.beta1;
  a.b2 = c->cfg.beta2;
  a.eps = c->cfg.epsilon;
  const bool tw = c->hnp && c->wtw_ok;
  a.tw = tw ? c->wtw : nullptr;
  a.tps = (long long)c->L.total;
  a.tnp = c->hnp;
  a.tt = soft ? c->target : nullptr;
  a.tau = c->cfg.tau;
  a.omt = (float)(1.0 - (double)c->cfg.tau);
  a.ttw = (soft && tw) ? c->wtw + (size_t)c->hnp * c->L.total : nullptr;
  a.hk = adam_hooks_for(c, net, soft);
  {
    ProfScope ps(c, soft ? "adam+reduce+soft_update" : "adam+reduce", 0,
                 (soft ? 40.0 : 28.0) * n + rbytes);
    hipLaunchKernelGGL(adam_reduce_kernel, dim3(blocks), dim3(256), 0, c->cur, t, a);
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
// Narrow weight gradients fused into a dX epilogue (GemmEpi.nw_*, gemm_common.h):
// dW1 = s^T dz1 from the dz1 GEMM, dWs = s^T dcat_s and dWa = a^T dcat_a from
// the dcat GEMM -- the tile's final values times the narrow operand's rows,
// one fp32 partial per 128-row tile (and row group), summed by grad_reduce.
// Replaces the skinny launches and the writes of dz1 / dcat nobody else reads.
// Needs the dX on gemm_h3 / gemm_h3m (one-pass epilogue: fp32 contexts on the
// twin path), whole 128-row and 128-column tiles, a <= 64-wide narrow side.
static int nw_rg(int K) { return std::max(1, 16 / ((K + 3) / 4)); }
static bool nw_ok(ddpg_ctx* c, const float* dx_a, int ld_a, const float* dx_b, int ld_b, int B,
                  int N, int Kd, const float* x, int ldx, int K, const float* buf) {
  int kh;
  return buf && c->sw.nw_fuse && c->sw.gemm_h3 &&
         ((c->hnp == 3 && B % 128 == 0) || (c->hnp == 1 && B % 256 == 0)) &&
         N % 128 == 0 && K >= 1 && K <= 64 && ldx % 4 == 0 && ((K + 3) & ~3) <= ldx &&
         aligned16(x) && gemm_h_ok<L_RK, L_RK>(c, dx_a, ld_a, dx_b, ld_b, B, N, Kd, 1, &kh);
}
static void nw_set(GemmEpi& e, int set, const float* x, int ldx, int K, float* out, int ld) {
  e.nw_x[set] = x;
  e.nw_ldx[set] = ldx;
  e.nw_k[set] = K;
  e.nw_ld[set] = ld;
  e.nw_rg[set] = nw_rg(K);
  e.nw_out[set] = out;
  e.nw_slab[set] = (long long)K * ld;
}

// in_window: work issued on the compute stream while the critic's exchange
// is in flight, before Adam waits for it (the fused data-parallel step puts
// the online actor forward there: it reads no critic parameter)
static void critic_train_dev(ddpg_ctx* c, int B, float inv_b, bool fused, int nq = -1,
                             bool par = false,
                             const std::function<void()>& in_window = std::function<void()>()) {
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
  // dWs / dWa in the same epilogue when they qualify (nw_ok); dcat is then
  // written only for a half whose weight gradient still reads it
  const float* whp = P(c, c->theta, L.c[CWH]);
  const bool fs = nw_ok(c, c->dhp, c->ldCH2, whp, c->CH2, B, 2 * c->CH1, c->CH2, c->s, c->ldS,
                        c->S, c->nw_Ws) &&
                  c->CH1 % 128 == 0;
  const bool fa = nw_ok(c, c->dhp, c->ldCH2, whp, c->CH2, B, 2 * c->CH1, c->CH2, c->a, c->ldA,
                        c->A, c->nw_Wa) &&
                  c->CH1 % 128 == 0;
  // each set owns its half's columns (nw_col1 = CH1 whenever either is
  // fused), so a state-only fusion never runs set 0 over the action half
  if (fs) nw_set(e, 0, c->s, c->ldS, c->S, c->nw_Ws, c->CH1);
  if (fa) nw_set(e, 1, c->a, c->ldA, c->A, c->nw_Wa, c->CH1);
  if (fs || fa) e.nw_col1 = c->CH1;
  if (fs && fa) e.out = nullptr;
  // one bf16 plane and dWs on the twin GEMM (S > 64, not the skinny kernel):
  // the state half's fp32 values have no reader -- only the action half
  // (dWa on the skinny kernel) is stored in fp32
  // (and with dWa fused above, no fp32 half has a reader: the twin alone)
  if (c->hnp == 1 && c->sw.half_twin && c->S > 64 /* SK_NMAX */ && act_twin(c, c->dcat).p &&
      gemm_h_ok<L_KR, L_KR>(c, c->s, c->ldS, c->dcat, c->ldC, c->S, c->CH1, B, 0, &kh)) {
    e.out_col0 = c->CH1;
    if (fa && !fs) {
      const Twin t = act_twin(c, c->dcat);
      e.outh = t.p;
      e.h_plane_stride = t.ps;
      e.h_planes = c->hnp;
      e.out = nullptr;
    }
  }
  GemmPlan pdc = gemm_launch<L_RK, L_RK>(c, "dx", c->dhp, c->ldCH2, P(c, c->theta, L.c[CWH]),
                                         c->CH2, B, 2 * c->CH1, c->CH2, e);
  const int mt = pdc.mt(B);
  // dWs = s^T . dcs ; dWa = a^T . dca  (unless fused above)
  GemmPlan pWs, pWa;
  if (!fs)
    pWs = wgrad_launch(c, c->s, c->ldS, c->dcat, c->ldC, c->S, c->CH1, B, c->slab_Ws,
                       c->split_cap_Ws, c->grad + L.c[CWS].off);
  if (!fa)
    pWa = wgrad_launch(c, c->a, c->ldA, c->dcat + c->CH1, c->ldC, c->A, c->CH1, B, c->slab_Wa,
                       c->split_cap_Wa, c->grad + L.c[CWA].off);
  if (par) fork_to(c, 5, c->aux[0], main);  // join dWh
  // gather every critic gradient into the flat grad buffer
  ReduceTable tab;
  tab.nseg = 0;
  const long long nWs = (long long)c->S * c->CH1, nWa = (long long)c->A * c->CH1;
  // the fused partials: one per 128 batch rows and row group (gemm_common.h)
  if (fs)
    add_seg(tab, c->nw_Ws, G + L.c[CWS].off, nWs, (B / 128) * nw_rg(c->S), nWs);
  else
    add_wgrad(tab, pWs, c->slab_Ws, G + L.c[CWS].off, nWs);
  add_seg(tab, c->colpart, G + L.c[CBS].off, 2 * c->CH1, mt, c->CH1);
  if (fa)
    add_seg(tab, c->nw_Wa, G + L.c[CWA].off, nWa, (B / 128) * nw_rg(c->A), nWa);
  else
    add_wgrad(tab, pWa, c->slab_Wa, G + L.c[CWA].off, nWa);
  add_seg(tab, c->colpart + c->CH1, G + L.c[CBA].off, 2 * c->CH1, mt, c->CH1);
  if (!c->comm) add_wgrad(tab, pWh, c->slab_Wh, G + L.c[CWH].off, nWh);
  add_seg(tab, part_dbh, G + L.c[CBH].off, c->CH2, nchunk, c->CH2);
  add_seg(tab, part_dWo, G + L.c[CWO].off, c->CH2, nchunk, c->CH2);
  add_seg(tab, part_dbo, G + L.c[CBO].off, 1, nchunk, 1);
  if (!c->comm) {
    adam_reduce_launch(c, 1, tab, !fused, fused);
    return;
  }
  reduce_launch(c, "grad_reduce", tab);
  if (c->comm) {
    // the rest of the critic ([Ws bs Wa ba] and [bh Wo bo]) behind dWh on the
    // comm stream, then the stats; Adam waits for all of it
    allreduce_on_cs(c, 1, "rccl_allreduce", G + L.critic_begin, L.c[CWH].off - L.critic_begin,
                    G + L.c[CBH].off, L.critic_end - L.c[CBH].off, true, "xwin|critic_tail");
    stats_allreduce_on_cs(c, true);
    if (in_window) in_window();
    join_cs(c, 2);
  } else if (in_window) {
    in_window();
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
  // dW3 = h2^T . dz3: in the dz2 thin_k launch below, which reads both (fw3,
  // TkPart.dw), or on its own (the skinny kernel)
  const bool fw3 = c->tk_dW3 && c->sw.nw_fuse;
  GemmPlan pW3;
  if (!fw3) {
    if (par) {
      fork_to(c, 6, main, c->aux[0]);
      c->cur = c->aux[0];
    }
    pW3 = wgrad_launch(c, c->h2, c->ldAH2, c->dz3, c->ldA, c->AH2, c->A, B, c->slab_W3,
                       c->split_cap_W3, G + L.a[AW3].off);
  }
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
  if (fw3) {
    tp.dw = c->tk_dW3;
    tp.dw_k = c->A;
    tp.dw_slab = (long long)c->AH2 * c->A;
  }
  bool w3_fused = false;
  int mt2 = thin_k_launch(c, "dx", &tp, 1, B, &w3_fused);
  if (fw3 && !w3_fused)
    pW3 = wgrad_launch(c, c->h2, c->ldAH2, c->dz3, c->ldA, c->AH2, c->A, B, c->slab_W3,
                       c->split_cap_W3, G + L.a[AW3].off);
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
  // dz1 = (dz2 . W2^T) * elu'(h1); colsum -> db1; dW1 = s^T dz1 in the same
  // epilogue when it qualifies (nw_ok: dz1 then has no reader and is not written)
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
  const float* w2p = P(c, c->theta, L.a[AW2]);
  const bool f1 = nw_ok(c, c->dz2, c->ldAH2, w2p, c->AH2, B, c->AH1, c->AH2, c->s, c->ldS, c->S,
                        c->nw_W1);
  if (f1) {
    nw_set(e, 0, c->s, c->ldS, c->S, c->nw_W1, c->AH1);
    e.out = nullptr;
    e.outh = nullptr;
  }
  GemmPlan pz1 = gemm_launch<L_RK, L_RK>(c, "dx", c->dz2, c->ldAH2, w2p, c->AH2, B, c->AH1,
                                         c->AH2, e);
  // dW1 = s^T . dz1  (unless fused above)
  GemmPlan pW1;
  if (!f1)
    pW1 = wgrad_launch(c, c->s, c->ldS, c->dz1, c->ldAH1, c->S, c->AH1, B, c->slab_W1,
                       c->split_cap_W1, G + L.a[AW1].off);
  if (par) fork_to(c, 3, c->aux[0], main);  // join dW3, dW2
  ReduceTable tab;
  tab.nseg = 0;
  const long long nW1 = (long long)c->S * c->AH1;
  if (f1)
    add_seg(tab, c->nw_W1, G + L.a[AW1].off, nW1, (B / 128) * nw_rg(c->S), nW1);
  else
    add_wgrad(tab, pW1, c->slab_W1, G + L.a[AW1].off, nW1);
  add_seg(tab, colpart1, G + L.a[AB1].off, c->AH1, pz1.mt(B), c->AH1);
  if (!c->comm) add_wgrad(tab, pW2, c->slab_W2, G + L.a[AW2].off, nW2);
  add_seg(tab, c->colpart, G + L.a[AB2].off, c->AH2, mt2, c->AH2);
  if (w3_fused)
    add_seg(tab, c->tk_dW3, G + L.a[AW3].off, (long long)c->AH2 * c->A, mt2,
            (long long)c->AH2 * c->A);
  else
    add_wgrad(tab, pW3, c->slab_W3, G + L.a[AW3].off, (long long)c->AH2 * c->A);
  if (!c->comm) {
    adam_reduce_launch(c, 0, tab, !fused, fused);
    return;
  }
  reduce_launch(c, "grad_reduce", tab);
  {  // [W1 b1] and [b2 W3] behind dW2 on the comm stream
    allreduce_on_cs(c, 4, "rccl_allreduce", G + L.actor_begin, L.a[AW2].off - L.actor_begin,
                    G + L.a[AB2].off, L.actor_end - L.a[AB2].off, false, "xwin|actor_tail");
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
  if (thin_k_launch(c, "fwd_l1", tp, TK_MAXP, B)) return true;
  // S > 64 (the bf16 configuration C5: S = 376): each part on thin_k where
  // it takes it, the rest as ONE gemm_h16i_pack_kernel launch (gemm_flush)
  if (!(c->hnp == 1 && c->sw.gemm_h3)) return false;
  c->gemm_defer = 1;
  for (int i = 0; i < TK_MAXP; ++i) {
    if (thin_k_launch(c, "fwd_l1", &tp[i], 1, B)) continue;
    GemmEpi e = epi_none();
    e.out = tp[i].out;
    e.outh = tp[i].outh;
    e.h_plane_stride = tp[i].hps;
    e.h_planes = c->hnp;
    e.ldo = tp[i].ldo;
    e.bias = tp[i].bias;
    e.act = tp[i].act;
    gemm_launch<L_RK, L_KR>(c, "fwd_l1", tp[i].X, tp[i].ldx, tp[i].W, tp[i].ldw, B, tp[i].N,
                            tp[i].K, e);
  }
  c->gemm_defer = 0;
  gemm_flush(c);
  return true;
}

static void learner_step_dev(ddpg_ctx* c, int B, float inv_b) {
  const hipStream_t s0 = c->cur;
  const hipStream_t s1 = c->par ? c->aux[0] : s0, s2 = c->par ? c->aux[1] : s0;
  // ddpg.py:90-109's batch-only first layers, all at once (every later use
  // reads them with the same pre-step parameters)
  const bool l1 = first_layers_dev(c, B);
  const bool mu_in_window = c->comm && !c->par;
  if (l1 && !c->par && !mu_in_window && c->sw.fwd_pack) {
    // The three layers that read only the first layers' outputs -- target
    // actor W2 (ddpg.py:90), online actor W2 (ddpg.py:106) and online critic
    // Wh (ddpg.py:100) -- as ONE pack launch (gemm_flush: a CU starts the next
    // part's tile while the previous tile's epilogue drains), then what
    // depends on them.  Same buffers, same per-tile arithmetic as the
    // sequential order below (DDPG_FWD_PACK=0): bitwise equal.
    c->gemm_defer = 1;
    std::swap(c->ppart, c->ppart_t);
    const GemmPlan pt = actor_l2(c, c->target, B, c->th1, nullptr);
    std::swap(c->ppart, c->ppart_t);
    const GemmPlan po = actor_l2(c, c->theta, B, c->h1, c->h2);
    const int nq = critic_fwd(c, c->theta, c->s, c->a, B, c->cat, c->h, 0, nullptr, 2);
    c->gemm_defer = 0;
    gemm_flush(c);
    // mu' = actor.predict_target(s2), then critic.predict_target(s2, mu')
    std::swap(c->ppart, c->ppart_t);
    std::swap(c->qpart, c->qpart_t);
    actor_out_launch(c, pt.nt(c->AH2), B, nullptr, c->ta2);
    c->td_nqt = critic_fwd(c, c->target, c->s2, c->ta2, B, c->tcat, nullptr, 1, nullptr, 1);
    std::swap(c->ppart, c->ppart_t);
    std::swap(c->qpart, c->qpart_t);
    actor_out_launch(c, po.nt(c->AH2), B, c->o, c->mu);  // a_outs (ddpg.py:106)
    critic_train_dev(c, B, inv_b, true, nq, false);
    critic_action_grad(c, c->s, c->mu, B, nullptr, c->dz3, c->o);
    actor_train_dev(c, B, true, false);
    return;
  }
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
  // a_outs = actor.predict(s)  ddpg.py:106 (actor params are unchanged until
  // actor.train).  Data-parallel step on one stream: issued inside the
  // critic's exchange window instead (it reads no critic parameter), so the
  // critic's tail all-reduce runs under it rather than in front of Adam.
  auto online_actor_fwd = [&] { actor_fwd(c, c->theta, c->s, B, c->h1, c->h2, c->o, c->mu, l1); };
  if (!mu_in_window) {
    c->cur = s2;
    online_actor_fwd();
  }
  // critic.train(s, a, y)  ddpg.py:100: forward now, loss once y is ready
  c->cur = s0;
  const int nq = critic_fwd(c, c->theta, c->s, c->a, B, c->cat, c->h, 0, nullptr, l1 ? 2 : 0);
  fork_to(c, 1, s1, s0);  // join target path (y)
  if (mu_in_window)
    critic_train_dev(c, B, inv_b, true, nq, c->par, online_actor_fwd);
  else
    critic_train_dev(c, B, inv_b, true, nq, c->par);
  // grads = critic.action_gradients(s, a_outs)  ddpg.py:107 (updated critic)
  fork_to(c, 2, s2, s0);  // join online actor forward (h1, h2, o, mu)
  critic_action_grad(c, c->s, c->mu, B, nullptr, c->dz3, c->o);
  // actor.train(s, grads[0])  ddpg.py:109  (forward above reused: same params)
  actor_train_dev(c, B, true, c->par);
  // actor/critic.update_target_network()  ddpg.py:112-113 and both Adam power
  // updates (_finish): done inside the two Adam passes above (AdamHooks)
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
  // each role's workgroups on one XCD (one L2 streams the weights) while they
  // fit its 32 CUs: +3 % at C2 (profiles/r3/sb_xcd_ab_c2.txt); phase 1's
  // three roles take XCDs 0, 1, 2
  a.xstride = c->sb_xstride ? c->sb_xstride : (ceil_div(B, SB_R) <= 32 ? 8 : 1);
  return a;
}

// Small-batch learner step: 4 launches (small_batch.h); the gather from the
// replay ring is fused into the phase kernels (slots already in c->d_slots).
// With a communicator (data parallelism at the reference's own batch sizes,
// parameters.py:11,32-34: each rank gathers its slice of the global draw)
// each network's gradient / Adam kernel runs as two launches around the RCCL
// sum of that network's flat gradient range: 6 launches + 2 exchanges (the
// critic's with the stats all-gather), each Adam waiting for its exchange.
static void sb_wgrad(ddpg_ctx* c, const SbArgs& a, int net, int G, int mode, double nflat) {
  ProfScope ps(c, mode == 2 ? "sb_adam" : "sb_wgrad_adam", mode == 2 ? 0.0 : 2.0 * a.B * nflat,
               32.0 * nflat);
  const SbGradTab& t = c->sb_tab[net];
  hipLaunchKernelGGL(sb_wgrad_adam_kernel, dim3(t.t[t.n].tile0), dim3(SB_GT), 0, c->cur, a, t,
                     net, G, mode);
  HIP_TRY(hipGetLastError());
}

static void learner_step_small(ddpg_ctx* c, ddpg_replay* rb, int B, float inv_b) {
  const Layout& L = c->L;
  const SbArgs a = sb_args(c, rb, B, inv_b);
  const int G = ceil_div(B, SB_R);
  const long long nc = (long long)(L.critic_end - L.critic_begin);
  const long long na = (long long)(L.actor_end - L.actor_begin);
  const double row_bytes = (2.0 * c->S + c->A + 2) * 4.0;
  const bool dp = c->comm != nullptr;
  float* const Gb = c->grad;
  {
    // three sets of workgroups: online critic rows (role 0: the online
    // critic and Wh^T), actor rows (1: the online actor), target rows (2: the
    // target actor and critic)
    ProfScope ps(c, "sb_phase1", 0,
                 4.0 * (double)G * (L.total + nc + na) + 2.0 * B * row_bytes);
    const int grid = a.xstride > 1 ? G * a.xstride : 3 * G;
    hipLaunchKernelGGL(sb_phase1_kernel, dim3(grid), dim3(SB_NT), c->sb_smem, c->cur, a);
    HIP_TRY(hipGetLastError());
  }
  if (!dp) {
    sb_wgrad(c, a, 1, G, 0, (double)nc);
  } else {
    sb_wgrad(c, a, 1, G, 1, (double)nc);
    allreduce_on_cs(c, 1, "rccl_allreduce", Gb + L.critic_begin, (size_t)nc, nullptr, 0, true,
                    nullptr);
    stats_allreduce_on_cs(c, true);
    join_cs(c, 2);
    sb_wgrad(c, a, 1, G, 2, (double)nc);
  }
  {
    ProfScope ps(c, "sb_phase3", 0,
                 4.0 * (double)G * (nc + (double)c->CH1 * c->CH2 + (double)c->AH1 * c->AH2) +
                     B * (c->S + c->A + c->AH1 + c->AH2) * 4.0);
    hipLaunchKernelGGL(sb_phase3_kernel, dim3(G * a.xstride), dim3(SB_NT), c->sb_smem, c->cur, a);
    HIP_TRY(hipGetLastError());
  }
  if (!dp) {
    sb_wgrad(c, a, 0, G, 0, (double)na);
  } else {
    sb_wgrad(c, a, 0, G, 1, (double)na);
    allreduce_on_cs(c, 4, "rccl_allreduce", Gb + L.actor_begin, (size_t)na, nullptr, 0, false,
                    nullptr);
    join_cs(c, 5);
    sb_wgrad(c, a, 0, G, 2, (double)na);
  }
}

static void gather_launch(ddpg_ctx* c, ddpg_replay* rb, int B);

// The fused learner step on this step's slots (c->d_slots): the small-batch
// path (gather fused) or gather + the large-batch GEMM path.
// world > 1 needs the communicator's exchange (a world > 1 ctx without one
// -- the rank-slice tests -- stays on the large path, whose unexchanged
// gradients are that rank's partial sums)
static bool takes_small(const ddpg_ctx* c, int B) {
  return c->sb_ok && (c->world == 1 || c->comm) && B <= c->sb_max_b;
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
  if (c->sw.stats_spin && (size_t)B * cols <= kRowsInMax) {
    // small rows (the 1:1 methods at small batch) in the kernel arguments
    RowsIn in;
    memcpy(in.v, src, sizeof(float) * B * cols);
    hipLaunchKernelGGL(rows_in_kernel, dim3(1), dim3(256), 0, c->stream, in, dst, ld, B, cols);
    HIP_TRY(hipGetLastError());
  } else {
    HIP_TRY(hipMemcpy2DAsync(dst, (size_t)ld * 4, src, (size_t)cols * 4, (size_t)cols * 4, B,
                             hipMemcpyHostToDevice, c->stream));
  }
  const Twin t = act_twin(c, dst);
  if (t.p) {  // the twin covers the padded rows (pads are zero in both)
    hipLaunchKernelGGL(twin_kernel, dim3(std::min(ceil_div(B * ld, 256), 2048)), dim3(256), 0,
                       c->stream, dst, (long long)B * ld, t.p, t.ps, c->hnp);
    HIP_TRY(hipGetLastError());
  }
}
static void wait_words(ddpg_ctx* c, const volatile unsigned* w, int n, unsigned seq);
static unsigned next_seq(unsigned& s);
constexpr int kRowsOutMax = 4096;  // floats: small results through pinned memory
static void download_rows(ddpg_ctx* c, float* dst, const float* src, int ld, int B, int cols) {
  if (B <= 0 || cols <= 0) return;
  if (c->sw.stats_spin && (size_t)B * cols <= kRowsOutMax) {
    if (!c->h_rows_word) {
      HIP_TRY(hipHostMalloc(&c->h_rows_word, (16 + kRowsOutMax) * sizeof(unsigned),
                            hipHostMallocCoherent));
      memset(c->h_rows_word, 0, 16 * sizeof(unsigned));
    }
    const unsigned seq = next_seq(c->rows_seq);
    float* out = reinterpret_cast<float*>(c->h_rows_word + 16);
    hipLaunchKernelGGL(rows_out_kernel, dim3(1), dim3(256), 0, c->stream, src, ld, B, cols, out,
                       c->h_rows_word, seq);
    HIP_TRY(hipGetLastError());
    wait_words(c, c->h_rows_word, 1, seq);
    memcpy(dst, out, sizeof(float) * B * cols);
    return;
  }
  HIP_TRY(hipMemcpy2DAsync(dst, (size_t)cols * 4, src, (size_t)ld * 4, (size_t)cols * 4, B,
                           hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
}

static void check_b(ddpg_ctx* c, int B) {
  if (B <= 0 || B > c->Bmax) throw einval("batch %d outside [1, %d]", B, c->Bmax);
}

// Wait until every word w[0 .. n) reads seq (written by a kernel on c->stream
// after a system-scope release).  The kernel may queue behind asynchronous
// work: after 50 ms fall back to the stream wait, which also surfaces a fault.
static void wait_words(ddpg_ctx* c, const volatile unsigned* w, int n, unsigned seq) {
  const auto t0 = std::chrono::steady_clock::now();
  int b = 0;
  while (b < n) {
    if (w[b] == seq) {
      ++b;
      continue;
    }
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) {
      HIP_TRY(hipStreamSynchronize(c->stream));
      for (; b < n; ++b)
        if (w[b] != seq) throw einval("completion word %d never written", b);
      break;
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);
}

static unsigned next_seq(unsigned& s) {
  if (++s == 0) s = 1;  // 0 is the words' initial value
  return s;
}

static void stats_words_alloc(ddpg_ctx* c) {
  if (!c->h_stats_word) {
    HIP_TRY(hipHostMalloc(&c->h_stats_word, 4 * sizeof(unsigned), hipHostMallocCoherent));
    memset(c->h_stats_word, 0, 4 * sizeof(unsigned));
  }
}

// ddpg_sync: a completion word after the queued work, polled (the stream
// wait with DDPG_STATS_SPIN=0)
void sync_stream(ddpg_ctx* c) {
  if (!c->sw.stats_spin) {
    HIP_TRY(hipStreamSynchronize(c->stream));
    return;
  }
  stats_words_alloc(c);
  const unsigned seq = next_seq(c->stats_seq);
  hipLaunchKernelGGL(word_kernel, dim3(1), dim3(64), 0, c->stream, c->h_stats_word, seq);
  HIP_TRY(hipGetLastError());
  wait_words(c, c->h_stats_word, 1, seq);
}

// The stats (q_max, loss) of the work queued so far, synchronously.
static void read_stats(ddpg_ctx* c, float st[2]) {
  if (c->sw.stats_spin) {
    stats_words_alloc(c);
    const unsigned seq = next_seq(c->stats_seq);
    float* out = reinterpret_cast<float*>(c->h_stats_word + 1);
    hipLaunchKernelGGL(stats_out_kernel, dim3(1), dim3(64), 0, c->stream, c->dstats, out,
                       c->h_stats_word, seq);
    HIP_TRY(hipGetLastError());
    wait_words(c, c->h_stats_word, 1, seq);
    st[0] = out[0];
    st[1] = out[1];
    return;
  }
  HIP_TRY(hipMemcpyAsync(st, c->dstats, 2 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
}

// ddpg_create's small-batch part (small_batch.h): whether the dims fit the
// phase kernels' LDS budget, the saved-tensor layout, the weight-gradient
// tables and the W^T shadows.  world > 1 never takes the small path.
void sb_setup(ddpg_ctx* c) {
  const int hmax = std::max(std::max(c->AH1, c->AH2), std::max(c->CH1, c->CH2));
  const int LX = rup(std::max(c->S, c->A), 4);
  const int LW = rup(std::max(std::max(c->AH1, c->AH2), std::max(2 * c->CH1, c->CH2)), 4);
  const size_t smem = sb_smem_floats(LX, LW) * sizeof(float);
  // vector weight streams need 4-aligned widths; 160 KiB of LDS per workgroup
  // (any world: takes_small sends a world > 1 ctx here only with a communicator)
  bool ok = hmax <= SB_MAXH && c->AH1 % 4 == 0 && c->AH2 % 4 == 0 &&
            c->CH1 % 4 == 0 && c->CH2 % 4 == 0 && smem <= 160 * 1024;
  if (const char* sv = getenv("DDPG_SMALL")) ok = ok && atoi(sv) != 0;
  if (ok) {
    c->sb_max_b = std::min(c->Bmax, SB_MAXB);
    c->sb_smem = smem;
    if (const char* xv = getenv("DDPG_SB_XCD")) c->sb_xstride = atoi(xv) ? 8 : 1;
    const size_t Bp = (size_t)rup(c->sb_max_b, 4);
    // saved tensors, feature-major [width][Bp]:
    // xs xa cat dcat h dhp q h1 h2 dz1 dz2 dz3 o y
    const size_t widths[14] = {(size_t)c->S, (size_t)c->A, 2 * (size_t)c->CH1,
                               2 * (size_t)c->CH1, (size_t)c->CH2, (size_t)c->CH2, 1,
                               (size_t)c->AH1, (size_t)c->AH2, (size_t)c->AH1,
                               (size_t)c->AH2, (size_t)c->A, (size_t)c->A, 1};
    size_t tot = 0;
    for (size_t w : widths) tot += (Bp * w + 63) / 64 * 64;
    HIP_TRY(hipMalloc(&c->sb_save, tot * sizeof(float)));
    HIP_TRY(hipMemset(c->sb_save, 0, tot * sizeof(float)));
    float* ptrs[14];
    size_t off = 0;
    for (int k = 0; k < 14; ++k) {
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
    sv.q = ptrs[6];
    sv.h1 = ptrs[7];
    sv.h2 = ptrs[8];
    sv.dz1 = ptrs[9];
    sv.dz2 = ptrs[10];
    sv.dz3 = ptrs[11];
    sv.o = ptrs[12];
    sv.y = ptrs[13];
    const Layout& L = c->L;
    const int bp = (int)Bp;
    auto add = [bp](SbGradTab& t, const Tensor& ts, const float* X, const float* dY,
                    int sdq = 0) {
      SbGradT& e = t.t[t.n];
      e.sdq = sdq;
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
    // one action: dz1 / dz2 saved per unit dz3 (small_batch.h sb_actor_rows)
    const int a1 = c->A == 1;
    add(ta, L.a[AW1], sv.xs, sv.dz1, a1);
    add(ta, L.a[AB1], nullptr, sv.dz1, a1);
    add(ta, L.a[AW2], sv.h1, sv.dz2, a1);
    add(ta, L.a[AB2], nullptr, sv.dz2, a1);
    add(ta, L.a[AW3], sv.h2, a1 ? nullptr : sv.dz3, a1);
    close(ta);
    ta.shadow = 2;
    SbGradTab& tc = c->sb_tab[1];  // critic (networks.py:130-137)
    tc.n = 0;
    // (the saved dcat / dhp are per unit dQ; dQ itself formed in the kernel)
    add(tc, L.c[CWS], sv.xs, sv.dcat, 1);
    add(tc, L.c[CBS], nullptr, sv.dcat, 1);
    add(tc, L.c[CWA], sv.xa, sv.dcat + (size_t)c->CH1 * Bp, 1);
    add(tc, L.c[CBA], nullptr, sv.dcat + (size_t)c->CH1 * Bp, 1);
    add(tc, L.c[CWH], sv.cat, sv.dhp, 1);
    add(tc, L.c[CBH], nullptr, sv.dhp, 1);
    add(tc, L.c[CWO], sv.h, nullptr, 1);
    add(tc, L.c[CBO], nullptr, nullptr, 1);
    close(tc);
    tc.shadow = 4;
    HIP_TRY(hipMalloc(&c->sb_misc, 4 * sizeof(float)));
    HIP_TRY(hipMemset(c->sb_misc, 0, 4 * sizeof(float)));
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
    HIP_TRY(hipHostMalloc(&c->h_pred_done, SB_PRED_BLOCKS * sizeof(unsigned), hipHostMallocCoherent));
    memset(c->h_pred_done, 0, SB_PRED_BLOCKS * sizeof(unsigned));
    c->sb_ok = true;
  }
}

// ====================================================================== C ABI
extern "C" {

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
      const int nb = ceil_div(B, SB_R);
      const bool spin = c->sw.pred_spin && c->h_pred_done;
      const unsigned seq = next_seq(c->pred_seq);
      {
        ProfScope ps(c, "sb_actor_predict", 0, 0);
        hipLaunchKernelGGL(sb_actor_predict_kernel, dim3(nb), dim3(SB_NT), smem, c->stream, a,
                           target ? c->target : c->theta, in, c->h_pred,
                           spin ? c->h_pred_done : nullptr, seq);
        HIP_TRY(hipGetLastError());
      }
      if (spin)  // the blocks' completion words
        wait_words(c, c->h_pred_done, nb, seq);
      else
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
      read_stats(c, st);
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

// ---------------------------------------------------------------- fused step
static void gather_launch(ddpg_ctx* c, ddpg_replay* rb, int B) {
  ProfScope ps(c, "gather", 0, (double)B * (2.0 * c->S + c->A + 2) * 8.0);
  const Twin ts = act_twin(c, c->s), ts2 = act_twin(c, c->s2);
  if (c->sw.gather16 && !rb->rsd && c->S % 4 == 0 && c->S <= 512 && c->A <= 64 &&
      c->ldS % 4 == 0 && (ts.ps & 3) == 0 && (ts2.ps & 3) == 0) {
    auto k = c->S <= 64 ? gather_rows16_kernel<1> : gather_rows16_kernel<8>;
    hipLaunchKernelGGL(k, dim3(ceil_div(B, 16)), dim3(256), 0, c->cur,
                       c->slots_src ? c->slots_src : c->d_slots, B, rb->rs, rb->ra, rb->rr,
                       rb->rt, rb->rs2, c->S, c->A, c->s, c->s2, c->ldS, c->a, c->ldA, c->r,
                       c->t, c->has_scaler ? c->dmean : nullptr,
                       c->has_scaler ? c->dscale : nullptr, ts.p, ts2.p, ts.ps, c->hnp);
    HIP_TRY(hipGetLastError());
    return;
  }
  hipLaunchKernelGGL(gather_rows_kernel, dim3(ceil_div(B, 4)), dim3(256), 0, c->cur,
                     c->slots_src ? c->slots_src : c->d_slots, B, rb->rs, rb->ra, rb->rr, rb->rt,
                     rb->rs2, rb->rsd, rb->rs2d,
                     rb->rrd, c->S, c->A, c->s,
                     c->s2, c->ldS, c->a, c->ldA, c->r, c->t, c->has_scaler ? c->dmean : nullptr,
                     c->has_scaler ? c->dscale : nullptr, act_twin(c, c->s).p,
                     act_twin(c, c->s2).p, act_twin(c, c->s).ps, c->hnp);
  HIP_TRY(hipGetLastError());
}

// Every argument check of a fused step, before anything has a side effect: a
// rejected call leaves the replay's sampler, the parameters and the Adam
// state as they were.
static void check_step(ddpg_ctx* c, const ddpg_replay* rb, int Bg, bool sampled) {
  if (rb->S != c->S || rb->A != c->A)
    throw einval("replay dims (S=%d, A=%d) != network dims (S=%d, A=%d)", rb->S, rb->A, c->S,
                 c->A);
  if (Bg <= 0 || Bg % c->world) throw einval("global batch %d not divisible by world %d", Bg, c->world);
  check_b(c, Bg / c->world);
  if (sampled && rb->count < Bg)  // random.sample without replacement
    throw einval("replay holds %lld rows < batch %d", (long long)rb->count, Bg);
}

static void step_common(ddpg_ctx* c, ddpg_replay* rb, const int64_t* idx, int Bg,
                        ddpg_stats* stats) {
  // rows flushed asynchronously (replay_flush's kernel-argument form) land
  // before this step's gather
  if (rb->written_rec && rb->written_by != c->uid)
    HIP_TRY(hipStreamWaitEvent(c->stream, rb->written, 0));
  const int B = Bg / c->world;
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
  if (c->graph_auto == 2 && small) {
    idle = false;  // small path: always eager
  } else if (c->graph_auto && small) {
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
        // RCCL calls did not capture here: this ctx runs its steps eagerly.
        // The failed capture launched nothing (its collectives were only
        // recorded) and allreduce_on_cs closed its group, so the eager step
        // below issues the same collectives in the same order as a peer rank
        // replaying its graph.  Visible through ddpg_step_counts.
        c->comm_graph = false;
        c->graph_fail = 1;
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
      ++c->n_graph_steps;
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
    ++c->n_eager_steps;
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
    read_stats(c, st);
    stats->q_max = st[0];
    stats->loss = st[1];
  }
}

int ddpg_learner_step(ddpg_ctx* c, ddpg_replay* rb, int Bg, ddpg_stats* stats) {
  return guard(c, [&] {
    if (!rb) throw einval("null replay");
    replay_flush(rb, rb->device == c->cfg.device ? c->stream : nullptr, c->uid);
    check_step(c, rb, Bg, true);
    c->idx_tmp.resize(Bg);
    if (rb->sampler.sample(rb->count, Bg, c->idx_tmp.data()) != 0) throw einval("sample failed");
    step_common(c, rb, c->idx_tmp.data(), Bg, stats);
  });
}

int ddpg_learner_step_indices(ddpg_ctx* c, ddpg_replay* rb, const int64_t* idx, int Bg,
                              ddpg_stats* stats) {
  return guard(c, [&] {
    if (!rb || !idx) throw einval("null argument");
    replay_flush(rb, rb->device == c->cfg.device ? c->stream : nullptr, c->uid);
    check_step(c, rb, Bg, false);
    for (int i = 0; i < Bg; ++i)
      if (idx[i] < 0 || idx[i] >= rb->count) throw einval("index %lld out of range", (long long)idx[i]);
    step_common(c, rb, idx, Bg, stats);
  });
}

}  // extern "C"
