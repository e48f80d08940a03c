// C-ABI lifecycle (ddpg_create / destroy / sync), parameter I/O, stats
// readback, profiling and error reporting.  include/ddpg_hip.h.
#include <atomic>
#include "ctx.h"

thread_local std::string g_err;

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
  if (c->h_pred_done) (void)hipHostFree(c->h_pred_done);
  if (c->h_stats_word) (void)hipHostFree(c->h_stats_word);
  if (c->h_rows_word) (void)hipHostFree(c->h_rows_word);
  for (auto& g : c->gslot) {
    if (g.exec) (void)hipGraphExecDestroy(g.exec);
    if (g.h_idx) (void)hipHostFree(g.h_idx);
    if (g.done) (void)hipEventDestroy(g.done);
  }
  if (c->step_done) (void)hipEventDestroy(c->step_done);
  for (void* p : {(void*)c->sb_save, (void*)c->sb_misc, (void*)c->sb_whT, (void*)c->sb_w2T})
    if (p) (void)hipFree(p);
  for (void* p : {(void*)c->atw, (void*)c->wtw, (void*)c->kc_part, (void*)c->kc_ticket})
    if (p) (void)hipFree(p);
  for (void* p : {(void*)c->dparams, (void*)c->dpw, (void*)c->dact, (void*)c->d_slots,
                  (void*)c->dmean, (void*)c->dscale, (void*)c->dacc, (void*)c->dstats_all,
                  (void*)c->xbuf, (void*)c->xrs})
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
  static std::atomic<uint64_t> next_uid{1};
  c->uid = next_uid++;
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
    {  // thin_k's grid target: blocks resident at once (TK_LDS bytes of LDS each)
      int cus = 0, lds = 0;
      HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, k.device));
      HIP_TRY(hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor,
                                    k.device));
      c->tk_slots = std::max(1, cus) * std::max(1, lds / TK_LDS);
    }
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
    {
      auto env_is = [](const char* name, const char* val) {
        const char* v = getenv(name);
        return v && strcmp(v, val) == 0;
      };
      c->sw.gemm_h = !env_is("DDPG_GEMM_H", "0");
      c->sw.gemm_s3 = !env_is("DDPG_GEMM", "f32");
      c->sw.thin_k = !env_is("DDPG_THINK", "0");
      c->sw.gemm_h3 = !env_is("DDPG_GEMM_H3", "0");
      c->sw.gemm_m16 = !env_is("DDPG_GEMM_M16", "0");
      c->sw.nw_fuse = !env_is("DDPG_NW_FUSE", "0");
      if (const char* v = getenv("DDPG_GEMM256")) c->sw.gemm256 = atoi(v) == 1;
      if (const char* v = getenv("DDPG_GEMM_HW")) c->sw.gemm_hw = atoi(v) != 0;
      c->sw.xcd = env_is("DDPG_XCD", "0") ? 0 : 1;
      c->sw.xcd_rect = !env_is("DDPG_XCD_RECT", "0");
      c->sw.skinny = !env_is("DDPG_SKINNY", "0");
      c->sw.l1_batch = !env_is("DDPG_L1BATCH", "0");
      c->sw.act_planes = !env_is("DDPG_ACT32", "1");
      c->sw.slots_h2d = env_is("DDPG_SLOTS_H2D", "1");
      if (const char* v = getenv("DDPG_TK_RPB")) c->sw.tk_rpb = std::max(0, atoi(v));
      c->sw.kcomb = !env_is("DDPG_KCOMB", "0");
      c->sw.kc_wgrad = !env_is("DDPG_KCOMB_WGRAD", "0");
      c->sw.tk_fwd = !env_is("DDPG_TK_FWD", "0");
      c->sw.gemm_pack = !env_is("DDPG_GEMM_PACK", "0");
      c->sw.fwd_pack = !env_is("DDPG_FWD_PACK", "0");
      c->sw.gather16 = !env_is("DDPG_GATHER16", "0");
      c->sw.pred_spin = !env_is("DDPG_PRED_SPIN", "0");
      c->sw.stats_spin = !env_is("DDPG_STATS_SPIN", "0");
      c->sw.half_twin = !env_is("DDPG_HALF_TWIN", "0");
      c->sw.skinny_nl = !env_is("DDPG_SKINNY_NL", "0");
      c->sw.prof_shapes = env_is("DDPG_PROF_SHAPES", "1");
      if (const char* v = getenv("DDPG_KCOMB_BLOCKS"))
        c->sw.kc_blocks = std::min(kKcTickets, std::max(1, atoi(v)));
      if (const char* v = getenv("DDPG_KCOMB_SPLITS"))
        c->sw.kc_splits = std::min(KC_MAXS, std::max(2, atoi(v)));
      if (const char* v = getenv("DDPG_TEST_CS_SPIN")) c->test_cs_spin = std::max(0, atoi(v));
      if (env_is("DDPG_GRAPH_COMM", "0")) c->comm_graph = false;
    }
    if (const char* gv = getenv("DDPG_GRAPH")) c->use_graph = atoi(gv) != 0;
    if (const char* gv = getenv("DDPG_GRAPH_AUTO")) c->graph_auto = atoi(gv);
    if (const char* pv = getenv("DDPG_PAR")) c->par = atoi(pv) != 0;
    gemm_setup(c);  // split-K caps, small-M buffers, GEMM kernel attributes
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
    // the narrow weight gradients fused into the dX epilogues (twin contexts,
    // narrow side <= 64): one partial per 128 rows and row group
    if (c->hnp == 3 || c->hnp == 1) {
      const size_t mtm = (size_t)ceil_div(B, 128);
      auto rg = [](int k) { return (size_t)std::max(1, 16 / ((k + 3) / 4)); };
      if (c->S <= 64) {
        req.push_back({&c->nw_W1, mtm * rg(c->S) * c->S * c->AH1});
        req.push_back({&c->nw_Ws, mtm * rg(c->S) * c->S * c->CH1});
      }
      if (c->A <= 64) req.push_back({&c->nw_Wa, mtm * rg(c->A) * c->A * c->CH1});
      if (c->A <= 32)
        req.push_back({&c->tk_dW3, (size_t)ceil_div(B, TK_ROWS) * c->AH2 * c->A});
    }
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
    // the step's replay slots are read in place by the kernels (pinned host
    // memory, rewritten by the host kSlotRing steps later after slot_ev):
    // coherent, so a kernel never reads a GPU-cached copy of an older slot
    HIP_TRY(hipHostMalloc(&c->h_slots, kSlotRing * B * sizeof(int), hipHostMallocCoherent));
    for (int i = 0; i < kSlotRing; ++i) HIP_TRY(hipEventCreateWithFlags(&c->slot_ev[i], hipEventDisableTiming));
    c->idx_tmp.resize(B * c->world);
    for (auto& g : c->gslot) {
      HIP_TRY(hipHostMalloc(&g.h_idx, B * sizeof(int), hipHostMallocCoherent));
      HIP_TRY(hipEventCreateWithFlags(&g.done, hipEventDisableTiming));
    }
    HIP_TRY(hipEventCreateWithFlags(&c->step_done, hipEventDisableTiming));
    sb_setup(c);
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
  return guard(c, [&] { sync_stream(c); });
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

// ---------------------------------------------------------------- step mode
int ddpg_step_counts(ddpg_ctx* c, int64_t* graphed, int64_t* eager, int* capture_failed) {
  return guard(c, [&] {
    if (graphed) *graphed = c->n_graph_steps;
    if (eager) *eager = c->n_eager_steps;
    if (capture_failed) *capture_failed = c->graph_fail;
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
